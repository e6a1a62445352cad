"""GPU: PinnedTable (cudasp_amd/pinned.py) -- a tweak table copied once into
pinned host memory and scanned in place by the streaming kernel, with Arrow
list offsets (cudasp_stream_batch.output_lengths NULL) -- gives exactly
cudasp_scan_arrow's rows: the SQL file's queries, NULL rules and slices,
batch sizes that wrap the 64-entry descriptor ring, repeated scans of one
pinned table with different keys, the protocol variants, and the reference's
tweak-length error.  Every test runs on both implementations: PinnedTable
(Python publish loop) and NativePinnedTable (the C ABI cudasp_pinned_*,
csrc/host/pinned_table.cpp, fed Arrow runs through cudasp_pinned_append), in
both placements: pinned host memory (streaming kernels) and resident in HBM
(CUDASP_TABLE_HBM, k_scan_multi)."""
import pytest

import golden_io
from test_arrow_gpu import _arrow, _rows, _sql_table

pytestmark = pytest.mark.gpu
pa = pytest.importorskip("pyarrow")


@pytest.fixture(scope="module")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.fixture(params=["PinnedTable", "NativePinnedTable", "NativePinnedTable-hbm"])
def cls(request):
    import functools

    import cudasp_amd
    if request.param.endswith("-hbm"):
        return functools.partial(cudasp_amd.NativePinnedTable, placement="hbm")
    return getattr(cudasp_amd, request.param)


def _nbatches(pt):
    return pt.info()["batches"] if hasattr(pt, "info") else len(pt.batches)


def _keys(q):
    return bytes.fromhex(q["scan_key"]), bytes.fromhex(q["spend_key"]), [bytes.fromhex(l) for l in q["label_keys"]]


def test_sql_file_pinned(gpu, cls):
    from cudasp_amd import cudasp_scan_arrow
    sc = golden_io.load("sql_cases.json")
    for q in sc["queries"]:
        tbl = _arrow(_sql_table(sc, q))
        with cls(tbl, batch_size=q["batch_size"]) as pt:
            out = pt.scan(*_keys(q))
        assert _rows(out) == _rows(cudasp_scan_arrow(tbl, *_keys(q), batch_size=q["batch_size"])), q["line"]
        got = [out.num_rows] if q["select"] == "count" else sorted(out.column("height").to_pylist())
        assert got == q["expected"], (q["line"], got)


def test_nulls_slices_types(gpu, cls):
    from cudasp_amd import cudasp_scan_arrow
    sc = golden_io.load("sql_cases.json")
    q = sc["queries"][2]
    r = [x for x in sc["tables"]["test_data"] if x["height"] == 200][0]
    tw, txid, v = bytes.fromhex(r["tweak"]), bytes.fromhex(r["txid"]), r["outputs"][0]
    keys = (bytes.fromhex(q["scan_key"]), bytes.fromhex(q["spend_key"]), [])
    rows = [
        (txid, 1, tw, [v]), (None, 2, tw, [v]), (txid, None, tw, [v]), (txid, 4, None, [v]),
        (txid, 5, tw, None), (txid, 6, tw, [None, v]), (txid, 7, tw, []), (b"", 8, tw, [v, v]),
    ] * 50
    for tweak_type in (None, pa.binary(64)):
        for large in (False, True):
            if large and tweak_type is not None:
                continue
            tbl = _arrow(rows, tweak_type, large)
            for t in (tbl, tbl.slice(37, 250)):
                with cls(t, batch_size=64) as pt:
                    assert _rows(pt.scan(*keys)) == _rows(cudasp_scan_arrow(t, *keys))
    with cls(_arrow([]), batch_size=10) as pt:
        assert pt.scan(*keys).num_rows == 0


@pytest.mark.parametrize("batch_size", [1, 37, 2048, 300000])
def test_batches_ring_and_repeated_scans(gpu, cls, batch_size):
    """5120 random rows with planted base and label matches: at batch_size 1
    and 37 more than 64 batches pass the descriptor ring; one pinned table is
    scanned again with other keys and again with the first ones."""
    from cudasp_amd import cudasp_scan_arrow
    rr = golden_io.load("random_rows.json")
    rows = [(i.to_bytes(32, "big"), i, bytes.fromhex(x["tweak"]), x["outputs"]) for i, x in enumerate(rr["rows"])]
    tbl = _arrow(rows * 40 if batch_size > 1 else rows * 2)
    k1 = (bytes.fromhex(rr["scan_key"]), bytes.fromhex(rr["spend_key"]), [bytes.fromhex(l) for l in rr["label_keys"]])
    k2 = (k1[0], k1[1], [])
    want1 = _rows(cudasp_scan_arrow(tbl, *k1))
    want2 = _rows(cudasp_scan_arrow(tbl, *k2))
    assert want1 and want1 != want2
    with cls(tbl, batch_size=batch_size) as pt:
        assert _rows(pt.scan(*k1)) == want1
        assert _rows(pt.scan(*k2)) == want2
        assert _rows(pt.scan(*k1)) == want1
        assert pt.last_stats["matches"] == len(want1) and pt.last_stats["batches"] == _nbatches(pt)


def test_variants(gpu, cls):
    from cudasp_amd import cudasp_scan_arrow
    rr = golden_io.load("random_rows.json")
    rows = [(i.to_bytes(32, "big"), i, bytes.fromhex(x["tweak"]), x["outputs"]) for i, x in enumerate(rr["rows"])]
    tbl = _arrow(rows * 4)
    keys = (bytes.fromhex(rr["scan_key"]), bytes.fromhex(rr["spend_key"]), [bytes.fromhex(l) for l in rr["label_keys"]])
    with cls(tbl, batch_size=100) as pt:
        for oc, neg in ((2, None), (8, True), (None, True)):
            want = _rows(cudasp_scan_arrow(tbl, *keys, batch_size=100, output_count=oc, label_negation=neg))
            assert _rows(pt.scan(*keys, output_count=oc, label_negation=neg)) == want, (oc, neg)


def test_errors(gpu, cls):
    from cudasp_amd import CudaspError, InvalidInputException
    rr = golden_io.load("random_rows.json")
    with pytest.raises(CudaspError, match="64 bytes"):
        cls(_arrow([(b"t", 1, bytes.fromhex(rr["rows"][0]["tweak"]), [1]), (b"u", 2, b"\x01" * 63, [1])]))
    rows = [(b"t", 1, bytes.fromhex(rr["rows"][0]["tweak"]), [1])]
    with cls(_arrow(rows)) as pt:
        with pytest.raises(InvalidInputException):
            pt.scan(b"\x01" * 31, bytes.fromhex(rr["spend_key"]), [])


@pytest.mark.parametrize("devices,batch_size", [([0, 0], 37), ([0, 0, 0], 2048)])
def test_logical_gpus(gpu, cls, devices, batch_size):
    """Batches round-robin over 2 or 3 logical GPUs on the one card (each its
    own scanner and streaming kernel on a share of the wave slots; at
    batch_size 37 each stream's 64-entry ring wraps): the rows of one GPU."""
    from cudasp_amd import cudasp_scan_arrow
    rr = golden_io.load("random_rows.json")
    rows = [(i.to_bytes(32, "big"), i, bytes.fromhex(x["tweak"]), x["outputs"]) for i, x in enumerate(rr["rows"])]
    tbl = _arrow(rows * 40)
    keys = (bytes.fromhex(rr["scan_key"]), bytes.fromhex(rr["spend_key"]), [bytes.fromhex(l) for l in rr["label_keys"]])
    want = _rows(cudasp_scan_arrow(tbl, *keys))
    with cls(tbl, batch_size=batch_size, devices=devices) as pt:
        if hasattr(pt, "batches"):
            assert {b["lg"] for b in pt.batches} == set(range(len(devices)))
        else:
            assert pt.info()["batches"] >= len(devices)
        assert _rows(pt.scan(*keys)) == want
        assert _rows(pt.scan(*keys[:2], [])) == _rows(cudasp_scan_arrow(tbl, *keys[:2], []))


@pytest.mark.parametrize("placement", ["pinned", "hbm"])
@pytest.mark.parametrize("piece_rows", [1, 37, 5000])
def test_native_runs_and_numbers(gpu, piece_rows, placement):
    """The C table takes the rows as many appended runs (batches span runs;
    NULL rows skipped but numbered): scan_rows gives the matching rows'
    positions in the input, ascending, as the oracle-pinned Arrow path finds
    them."""
    from cudasp_amd import NativePinnedTable, cudasp_scan_arrow
    rr = golden_io.load("random_rows.json")
    rows = [(i.to_bytes(32, "big"), i, bytes.fromhex(x["tweak"]), x["outputs"]) for i, x in enumerate(rr["rows"])]
    rows = [r if i % 7 else (None,) + r[1:] for i, r in enumerate(rows * 2)]  # every 7th row skipped
    tbl = _arrow(rows)
    keys = (bytes.fromhex(rr["scan_key"]), bytes.fromhex(rr["spend_key"]), [bytes.fromhex(l) for l in rr["label_keys"]])
    want = _rows(cudasp_scan_arrow(tbl, *keys, batch_size=500))
    with NativePinnedTable(tbl, batch_size=500, piece_rows=piece_rows, placement=placement) as pt:
        idx = pt.scan_rows(*keys)
        inf = pt.info()
    assert idx.tolist() == sorted(set(idx.tolist())) and all(i % 7 for i in idx.tolist())
    assert inf["rows_appended"] == len(rows) and inf["rows_pinned"] == len(rows) - len(range(0, len(rows), 7))
    assert inf["batches"] == -(-inf["rows_pinned"] // 500) and inf["last_matches"] == len(idx)
    assert inf["placement"] == (1 if placement == "hbm" else 0) and inf["device_bytes"] > 0
    got = _rows(tbl.take(__import__("pyarrow").array(idx)).select([0, 1, 2]))
    assert got == want


@pytest.mark.parametrize("placement", ["pinned", "hbm"])
def test_native_early_close(gpu, monkeypatch, placement):
    """Batches closed early by the outputs word cap (the u32-offset guard,
    lowered by CUDASP_PINNED_TEST_MAX_WORDS): more than 64 small batches of
    uneven row counts, the ring wrapped, rows as the Arrow path's."""
    from cudasp_amd import NativePinnedTable, cudasp_scan_arrow
    monkeypatch.setenv("CUDASP_PINNED_TEST_MAX_WORDS", "40")
    rr = golden_io.load("random_rows.json")
    rows = [(i.to_bytes(32, "big"), i, bytes.fromhex(x["tweak"]), x["outputs"]) for i, x in enumerate(rr["rows"])]
    tbl = _arrow(rows * 8)
    keys = (bytes.fromhex(rr["scan_key"]), bytes.fromhex(rr["spend_key"]), [bytes.fromhex(l) for l in rr["label_keys"]])
    with NativePinnedTable(tbl, batch_size=1000, placement=placement) as pt:
        got = _rows(pt.scan(*keys))
        assert pt.info()["batches"] > 64
    assert got == _rows(cudasp_scan_arrow(tbl, *keys))


@pytest.mark.parametrize("output_count", [None, 3])
def test_hbm_many_labels(gpu, output_count):
    """The resident placement takes any label count (k_scan_multi; the
    streaming kernel's scratch bounds the pinned placement's) and the
    per-batch path of output_count > 1: 40 labels, rows as the Arrow path's."""
    from cudasp_amd import NativePinnedTable, cudasp_scan_arrow
    rr = golden_io.load("random_rows.json")
    rows = [(i.to_bytes(32, "big"), i, bytes.fromhex(x["tweak"]), x["outputs"]) for i, x in enumerate(rr["rows"])]
    tbl = _arrow(rows * 4)
    labels = [bytes.fromhex(l) for l in rr["label_keys"]]
    import bench
    labels = labels + bench.label_keys(40)[len(labels):]
    keys = (bytes.fromhex(rr["scan_key"]), bytes.fromhex(rr["spend_key"]), labels)
    want = _rows(cudasp_scan_arrow(tbl, *keys, batch_size=200, output_count=output_count))
    assert want
    with NativePinnedTable(tbl, batch_size=200, placement="hbm") as pt:
        assert _rows(pt.scan(*keys, output_count=output_count)) == want


def test_library_loaded_before_torch_cuda(gpu):
    """A fresh process whose first GPU call is the library's (a
    NativePinnedTable) can still use torch's GPU afterwards: the package
    loads torch's HIP runtime before the library (cudasp_amd/_native.py)."""
    import os
    import subprocess
    import sys
    probe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "probes",
                         "init_order.py")
    r = subprocess.run([sys.executable, probe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "torch tensor ok" in r.stdout, (r.stdout[-500:], r.stderr[-1500:])


def test_native_tables_scanned_concurrently(gpu):
    """Two C tables on one GPU (one pinned, one resident), each scanned from
    its own thread with different keys at the same time, three times over:
    every scan's rows as the Arrow path's (separate scanners and kernels;
    the library's error state is per thread)."""
    import threading

    from cudasp_amd import NativePinnedTable, cudasp_scan_arrow
    rr = golden_io.load("random_rows.json")
    rows = [(i.to_bytes(32, "big"), i, bytes.fromhex(x["tweak"]), x["outputs"]) for i, x in enumerate(rr["rows"])]
    tbl = _arrow(rows * 20)
    k1 = (bytes.fromhex(rr["scan_key"]), bytes.fromhex(rr["spend_key"]), [bytes.fromhex(l) for l in rr["label_keys"]])
    k2 = (k1[0], k1[1], [])
    want = {0: _rows(cudasp_scan_arrow(tbl, *k1)), 1: _rows(cudasp_scan_arrow(tbl, *k2))}
    got, errors = {0: [], 1: []}, []
    tables = [NativePinnedTable(tbl, batch_size=700), NativePinnedTable(tbl, batch_size=900, placement="hbm")]
    try:
        def run(i):
            try:
                for _ in range(3):
                    got[i].append(_rows(tables[i].scan(*(k1 if i == 0 else k2))))
            except Exception as e:  # surfaced after join
                errors.append(e)
        ths = [threading.Thread(target=run, args=(i,)) for i in range(2)]
        for th in ths:
            th.start()
        for th in ths:
            th.join(timeout=120)
        assert not errors, errors
        assert got[0] == [want[0]] * 3 and got[1] == [want[1]] * 3
    finally:
        for t in tables:
            t.close()
