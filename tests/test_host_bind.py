"""CPU: bind-time validation of the C++ table-function host reproduces the
reference's InvalidInputException messages (src/cudasp_extension.cu:420-509)."""
import pytest

from cudasp_amd import BoundScan, InvalidInputException

SCAN = b"\x11" * 32
SPEND = b"\x22" * 64


def bind(*a, **k):
    return BoundScan(*a, **k)


def test_defaults():
    assert bind(SCAN, SPEND, []).batch_size == 300000
    assert bind(SCAN, SPEND, [SPEND], batch_size=50000).batch_size == 50000
    assert bind(SCAN, SPEND, [], batch_size=10_000_000).batch_size == 10_000_000


@pytest.mark.parametrize("args,kw,msg", [
    ((SCAN, SPEND, []), dict(arg_count=3),
     "cudasp_scan requires 4 arguments: TABLE, scan_private_key BLOB, spend_public_key BLOB, and label_keys LIST[BLOB]"),
    (("notblob", SPEND, []), {}, "Second argument must be a BLOB (32-byte scan_private_key)"),
    ((b"\x01" * 31, SPEND, []), {}, "scan_private_key must be exactly 32 bytes, got 31 bytes"),
    ((SCAN, 7, []), {}, "Third argument must be a BLOB (64-byte spend_public_key)"),
    ((SCAN, b"\x01" * 65, []), {}, "spend_public_key must be exactly 64 bytes, got 65 bytes"),
    ((SCAN, SPEND, b"x"), {}, "Fourth argument must be a LIST[BLOB] (label keys)"),
    ((SCAN, SPEND, [SPEND, 3]), {}, "All elements in label_keys must be BLOBs"),
    ((SCAN, SPEND, [SPEND, b"\x00" * 33]), {}, "Each label key must be exactly 64 bytes, got 33 bytes"),
    ((SCAN, SPEND, []), dict(batch_size="10"), "batch_size parameter must be an INTEGER"),
    ((SCAN, SPEND, []), dict(batch_size=0), "batch_size must be positive, got 0"),
    ((SCAN, SPEND, []), dict(batch_size=-5), "batch_size must be positive, got -5"),
    ((SCAN, SPEND, []), dict(batch_size=10_000_001), "batch_size too large (max 10,000,000), got 10000001"),
])
def test_bind_errors(args, kw, msg):
    with pytest.raises(InvalidInputException) as e:
        bind(*args, **kw)
    assert str(e.value) == msg


@pytest.mark.parametrize("k,msg", [
    (0, "output_count must be between 1 and 64, got 0"),
    (65, "output_count must be between 1 and 64, got 65"),
    (-3, "output_count must be between 1 and 64, got -3"),
])
def test_variant_parameter_errors(k, msg):
    """Named parameters of the protocol variants (cudasp_tf_bind_options)."""
    with pytest.raises(InvalidInputException) as e:
        bind(SCAN, SPEND, [], output_count=k)
    assert str(e.value) == msg
    assert bind(SCAN, SPEND, [], output_count=64, label_negation=True, full_x=True).full_x


def test_chunk_larger_than_a_vector_is_rejected():
    """A chunk may hold at most CUDASP_TF_VECTOR_SIZE rows: the batch slots
    are sized batch_size + one vector (include/cudasp_host.h), so a larger
    chunk is an argument error, raised before any GPU work."""
    import ctypes

    from cudasp_amd import _native
    from cudasp_amd import table_function as tf
    lib = tf._lib()
    bound = bind(SCAN, SPEND, [])
    g, loc = ctypes.c_void_p(), ctypes.c_void_p()
    assert lib.cudasp_tf_init(bound._h, ctypes.byref(g)) == 0
    assert lib.cudasp_tf_local_init(g, ctypes.byref(loc)) == 0
    try:
        keep, c = tf._make_chunk([(None, None, None, None)] * (tf.VECTOR_SIZE + 1))
        assert lib.cudasp_tf_function(bound._h, g, loc, ctypes.byref(c)) == _native.CUDASP_ERR_INVALID_ARG
        assert b"exceeds the vector size" in _native.load().cudasp_last_error()
    finally:
        lib.cudasp_tf_local_free(loc)
        lib.cudasp_tf_global_free(g)
