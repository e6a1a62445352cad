"""CPU: the Arrow-to-pinned-layout helpers of cudasp_amd.PinnedTable
(cudasp_amd/pinned.py) -- list offsets and values under the reference's NULL
rules (a NULL list is empty, NULL elements are dropped,
src/cudasp_extension.cu:195-221), slices, large types, and the 64-byte tweak
check."""
import numpy as np
import pytest

pa = pytest.importorskip("pyarrow")


def test_lists_null_rules_and_slices():
    from cudasp_amd.pinned import _lists
    a = pa.array([[1, 2], None, [3, None, 4], [], [5]], pa.list_(pa.int64()))
    offs, vals = _lists(a)
    assert offs.tolist() == [0, 2, 2, 4, 4, 5] and vals.tolist() == [1, 2, 3, 4, 5]
    offs, vals = _lists(a.slice(1, 3))
    assert offs.tolist() == [0, 0, 2, 2] and vals.tolist() == [3, 4]
    big = pa.array([[7, 8, 9], [10]], pa.large_list(pa.int64()))
    offs, vals = _lists(big)
    assert offs.tolist() == [0, 3, 4] and vals.tolist() == [7, 8, 9, 10]
    rng = np.random.default_rng(5)
    rows = [None if rng.random() < 0.1 else [None if rng.random() < 0.2 else int(x) for x in rng.integers(-9, 9, rng.integers(0, 6))]
            for _ in range(300)]
    offs, vals = _lists(pa.array(rows, pa.list_(pa.int64())))
    want = [[v for v in (r or []) if v is not None] for r in rows]
    assert [vals[offs[i]:offs[i + 1]].tolist() for i in range(len(rows))] == want


def test_blob64_types_and_errors():
    from cudasp_amd import CudaspError
    from cudasp_amd.pinned import _blob64
    rows = [bytes([i]) * 64 for i in range(5)]
    for t in (pa.binary(), pa.large_binary(), pa.binary(64)):
        a = pa.array(rows, t)
        assert (_blob64(a)[:, 0] == np.arange(5)).all()
        assert (_blob64(a.slice(2, 2))[:, 0] == [2, 3]).all()
    with pytest.raises(CudaspError, match="64 bytes"):
        _blob64(pa.array([bytes(64), bytes(63)], pa.binary()))


def test_native_pinned_table_fails_loudly_without_a_device():
    """The C pinned table (cudasp_pinned_create) checks batch_size like the
    bind and needs a GPU: no CPU fallback."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("device present")
    from cudasp_amd import CudaspError, InvalidInputException, NativePinnedTable, _native
    tbl = pa.table({"txid": pa.array([b"t"]), "height": pa.array([1], pa.int32()),
                    "tweak_key": pa.array([bytes(64)]), "outputs": pa.array([[1]], pa.list_(pa.int64()))})
    for bs, msg in ((0, "positive"), (10_000_001, "too large"), ("7", "INTEGER")):
        with pytest.raises(InvalidInputException, match=msg):
            NativePinnedTable(tbl, batch_size=bs)
    with pytest.raises(CudaspError) as e:
        NativePinnedTable(tbl)
    assert e.value.code == _native.CUDASP_ERR_NO_DEVICE


def _native_table(n, bad_tweak_at=None, outputs=2):
    rows_ok = [i % 7 != 0 for i in range(n)]
    return pa.table({
        "txid": pa.array([bytes([i % 256]) * 32 if rows_ok[i] else None for i in range(n)], pa.binary()),
        "height": pa.array(list(range(n)), pa.int32()),
        "tweak_key": pa.array([bytes(63) if i == bad_tweak_at else bytes([i % 256]) * 64 for i in range(n)]),
        "outputs": pa.array([None if i % 11 == 0 else [i] * outputs for i in range(n)], pa.list_(pa.int64())),
    })


@pytest.mark.parametrize("piece_rows", [1, 37, 1000])
def test_native_pinned_appends_without_a_device(monkeypatch, piece_rows):
    """cudasp_pinned_append's batching in the null-device mode (batches in
    plain host memory): NULL-txid rows skipped but counted, batches closed at
    batch_size across appended runs, and early when a batch's outputs would
    pass the word cap (CUDASP_PINNED_TEST_MAX_WORDS; 2^32 - 1 in the
    product); a run with a bad tweak keeps nothing; a scan fails loudly."""
    import ctypes

    from cudasp_amd import CudaspError, NativePinnedTable, _native
    from cudasp_amd.table_function import _PinnedInfo, _arrow_pieces, _columns, _lib
    monkeypatch.setenv("CUDASP_TF_NULL_DEVICE", "1")
    tbl = _native_table(1000)
    pinned = sum(1 for i in range(1000) if i % 7)
    with NativePinnedTable(tbl, batch_size=100, piece_rows=piece_rows) as pt:
        inf = pt.info()
        assert inf["rows_appended"] == 1000 and inf["rows_pinned"] == pinned
        assert inf["batches"] == -(-pinned // 100)
        with pytest.raises(CudaspError) as e:
            pt.scan(bytes(31) + b"\x01", bytes(64), [])
        assert e.value.code == _native.CUDASP_ERR_NO_DEVICE
    # early close: 2 outputs per row (none for NULL lists), at most 9 words per batch
    monkeypatch.setenv("CUDASP_PINNED_TEST_MAX_WORDS", "9")
    with NativePinnedTable(tbl, batch_size=100, piece_rows=piece_rows) as pt:
        words, nb = 0, 1
        for i in range(1000):
            if i % 7 == 0:
                continue
            w = 0 if i % 11 == 0 else 2
            if words + w > 9 and words > 0:
                nb, words = nb + 1, 0
            words += w
        assert pt.info()["batches"] == nb and pt.info()["rows_pinned"] == pinned
    monkeypatch.delenv("CUDASP_PINNED_TEST_MAX_WORDS")
    # a bad tweak in a later run: the earlier runs stay, nothing of that run
    with pytest.raises(CudaspError, match="64 bytes"):
        NativePinnedTable(_native_table(300, bad_tweak_at=250), batch_size=64, piece_rows=200)
    lib = _lib()
    h = ctypes.c_void_p()
    _native.check(lib.cudasp_pinned_create(64, None, 0, ctypes.byref(h)))
    try:
        pieces = _arrow_pieces(_native_table(300, bad_tweak_at=250), 200)
        _native.check(lib.cudasp_pinned_append(h, ctypes.byref(_columns(*pieces[0]))))
        assert lib.cudasp_pinned_append(h, ctypes.byref(_columns(*pieces[1]))) == _native.CUDASP_ERR_INVALID_ARG
        inf = _PinnedInfo()
        _native.check(lib.cudasp_pinned_info(h, ctypes.byref(inf)))
        assert inf.rows_appended == 200 and inf.rows_pinned == sum(1 for i in range(200) if i % 7)
    finally:
        lib.cudasp_pinned_free(h)


def test_native_pinned_argument_errors(monkeypatch):
    """cudasp_pinned_create_placed / _scan argument errors, loud and coded
    (null-device mode: no GPU needed): an unknown placement, batch_size above
    the bind's limit, an empty device list, and full_x at scan time."""
    import ctypes

    from cudasp_amd import _native
    from cudasp_amd.table_function import BoundScan, _lib
    monkeypatch.setenv("CUDASP_TF_NULL_DEVICE", "1")
    lib = _lib()
    h = ctypes.c_void_p()
    dev = (ctypes.c_int * 1)(0)
    assert lib.cudasp_pinned_create_placed(100, dev, 1, 5, ctypes.byref(h)) == _native.CUDASP_ERR_INVALID_ARG
    assert b"placement" in _native.load().cudasp_last_error()
    assert lib.cudasp_pinned_create_placed(10_000_001, dev, 1, 1, ctypes.byref(h)) == _native.CUDASP_ERR_INVALID_ARG
    assert b"too large" in _native.load().cudasp_last_error()
    assert lib.cudasp_pinned_create_placed(100, dev, 0, 0, ctypes.byref(h)) == _native.CUDASP_ERR_INVALID_ARG
    for placement in (0, 1):
        _native.check(lib.cudasp_pinned_create_placed(100, dev, 1, placement, ctypes.byref(h)))
        try:
            bound = BoundScan(bytes(31) + b"\x01", bytes(64), [], full_x=True)
            rows, count = ctypes.POINTER(ctypes.c_uint64)(), ctypes.c_uint64()
            assert lib.cudasp_pinned_scan(h, bound._h, ctypes.byref(rows), ctypes.byref(count)) == \
                _native.CUDASP_ERR_INVALID_ARG
            assert b"full_x" in _native.load().cudasp_last_error()
        finally:
            lib.cudasp_pinned_free(h)


@pytest.mark.parametrize("fail_at", [1, 2, 3])
def test_native_pinned_append_rolls_back_a_failed_close(monkeypatch, fail_at):
    """A batch close that fails inside cudasp_pinned_append (allocation or
    upload; forced here by CUDASP_PINNED_TEST_SEAL_FAIL) undoes the whole run:
    the counters return to their values before it, and retrying the run gives
    exactly the table appended without a failure -- no input number is handed
    out twice."""
    import ctypes

    from cudasp_amd import _native
    from cudasp_amd.table_function import _PinnedInfo, _arrow_pieces, _columns, _lib
    monkeypatch.setenv("CUDASP_TF_NULL_DEVICE", "1")
    lib = _lib()
    pieces = _arrow_pieces(_native_table(1000), 230)  # runs of 230 rows, batches of 100 (non-NULL rows)

    def info(h):
        inf = _PinnedInfo()
        _native.check(lib.cudasp_pinned_info(h, ctypes.byref(inf)))
        return (inf.rows_appended, inf.rows_pinned, inf.batches, inf.pinned_bytes)

    def build(fail):
        if fail:
            monkeypatch.setenv("CUDASP_PINNED_TEST_SEAL_FAIL", str(fail))
        else:
            monkeypatch.delenv("CUDASP_PINNED_TEST_SEAL_FAIL", raising=False)
        h = ctypes.c_void_p()
        _native.check(lib.cudasp_pinned_create(100, None, 0, ctypes.byref(h)))
        failed = 0
        for p in pieces:
            before = info(h)
            rc = lib.cudasp_pinned_append(h, ctypes.byref(_columns(*p)))
            if rc != _native.CUDASP_OK:
                assert rc == _native.CUDASP_ERR_CAPACITY and b"not appended" in _native.load().cudasp_last_error()
                assert info(h) == before
                failed += 1
                _native.check(lib.cudasp_pinned_append(h, ctypes.byref(_columns(*p))))  # the retry
        return h, failed

    ref, nf = build(0)
    got, failed = build(fail_at)
    try:
        assert nf == 0 and failed == 1
        assert info(got) == info(ref)
    finally:
        lib.cudasp_pinned_free(ref)
        lib.cudasp_pinned_free(got)
