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
