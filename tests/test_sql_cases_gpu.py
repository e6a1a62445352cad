"""GPU: every query of the reference's test/sql/cudasp.test through the C++
table-function host (bind -> per-thread accumulate -> batch -> GPU -> emit),
with the same tables, keys and batch sizes, several executor-thread counts;
results compared as multisets (the reference's output order is unspecified)."""
import pytest

import golden_io

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _table(sc, q):
    if q["table"] == "test_data":
        rows = sc["tables"]["test_data"][:q["test_data_rows_visible"]]
        rows = [r for r in rows if q["where_height"] in (None, r["height"])]
        return [(bytes.fromhex(r["txid"]), r["height"], bytes.fromhex(r["tweak"]), r["outputs"]) for r in rows]
    t = sc["tables"][q["table"]]
    r = t["row"]
    row = (bytes.fromhex(r["txid"]), r["height"], bytes.fromhex(r["tweak"]), r["outputs"])
    return [row] * t["repeat"]


@pytest.mark.parametrize("threads", [1, 3])
def test_sql_file(gpu, threads):
    from cudasp_amd import cudasp_scan
    sc = golden_io.load("sql_cases.json")
    for q in sc["queries"]:
        table = _table(sc, q)
        out = cudasp_scan(table, bytes.fromhex(q["scan_key"]), bytes.fromhex(q["spend_key"]),
                          [bytes.fromhex(l) for l in q["label_keys"]], batch_size=q["batch_size"], threads=threads)
        got = [len(out)] if q["select"] == "count" else sorted(h for _, h, _ in out)
        assert got == q["expected"], (q["line"], got)
        # emitted rows are the input rows verbatim
        ins = {(t, h, w) for t, h, w, _ in table}
        assert all(o in ins for o in out)


def test_nulls_and_edge_rows(gpu):
    """NULL txid/height/tweak rows are skipped, NULL outputs never match, NULL
    list elements are dropped (src/cudasp_extension.cu:195-221); empty input."""
    from cudasp_amd import cudasp_scan
    sc = golden_io.load("sql_cases.json")
    q = sc["queries"][2]  # BIP-352 vector keys; row 200 matches
    r = [x for x in sc["tables"]["test_data"] if x["height"] == 200][0]
    tw, txid = bytes.fromhex(r["tweak"]), bytes.fromhex(r["txid"])
    v = r["outputs"][0]
    keys = (bytes.fromhex(q["scan_key"]), bytes.fromhex(q["spend_key"]), [])
    table = [
        (txid, 1, tw, [v]),           # match
        (None, 2, tw, [v]),           # NULL txid: skipped
        (txid, None, tw, [v]),        # NULL height: skipped
        (txid, 4, None, [v]),         # NULL tweak: skipped
        (txid, 5, tw, None),          # NULL outputs: no match
        (txid, 6, tw, [None, v]),     # NULL element dropped, still matches
        (txid, 7, tw, []),            # empty list
        (b"", 8, tw, [v, v]),         # empty txid, duplicate outputs
    ]
    out = cudasp_scan(table, *keys)
    assert sorted(h for _, h, _ in out) == [1, 6, 8]
    assert cudasp_scan([], *keys) == []


def test_multi_batch_boundaries(gpu):
    """batch_size smaller than a chunk and not dividing it: every row still
    processed exactly once."""
    from cudasp_amd import cudasp_scan
    sc = golden_io.load("sql_cases.json")
    q = sc["queries"][0]
    t = sc["tables"]["large_test"]["row"]
    row = (bytes.fromhex(t["txid"]), t["height"], bytes.fromhex(t["tweak"]), t["outputs"])
    table = [row] * 5000
    for bs in (1, 7, 2048, 2049, 4999, 5000):
        out = cudasp_scan(table, bytes.fromhex(q["scan_key"]), bytes.fromhex(q["spend_key"]), [],
                          batch_size=bs, threads=2)
        assert len(out) == 5000, bs


def test_wrong_tweak_size_is_an_error(gpu):
    from cudasp_amd import CudaspError, cudasp_scan
    with pytest.raises(CudaspError):
        cudasp_scan([(b"t", 1, b"\x01" * 63, [1])], b"\x01" * 32, b"\x02" * 64, [])


def test_pooled_contexts_across_queries(gpu):
    """The host parks each thread's GPU state after a query and the next query
    reuses it with new keys (cudasp_scanner_set_keys): results must not
    depend on whether a context is fresh or pooled, including a change of the
    label count between queries."""
    from cudasp_amd import cudasp_scan, pool_size, release_pool
    sc = golden_io.load("sql_cases.json")
    release_pool()
    assert pool_size() == 0
    first = None
    for rnd in range(2):  # round 0 starts from an empty pool, round 1 from a warm one
        got = []
        for q in sc["queries"]:
            out = cudasp_scan(_table(sc, q), bytes.fromhex(q["scan_key"]), bytes.fromhex(q["spend_key"]),
                              [bytes.fromhex(l) for l in q["label_keys"]], batch_size=q["batch_size"], threads=2)
            got.append(sorted(out))
            assert pool_size() > 0
        if first is None:
            first = got
        assert got == first
    release_pool()
    assert pool_size() == 0


def test_scanner_set_keys(gpu):
    """A rebound scanner gives the same values as a fresh one."""
    import numpy as np
    import torch
    from cudasp_amd import Scanner
    rr = golden_io.load("random_rows.json")
    rows = rr["rows"][:256]
    scan, spend = bytes.fromhex(rr["scan_key"]), bytes.fromhex(rr["spend_key"])
    labels = [bytes.fromhex(l) for l in rr["label_keys"]]
    x, y = golden_io.tweak_columns(golden_io.tweak_array([r["tweak"] for r in rows]))
    n = len(rows)
    dx = torch.from_numpy(x.view(np.int32).copy()).cuda()
    dy = torch.from_numpy(y.view(np.int32).copy()).cuda()

    def values(s, nl):
        t = torch.zeros((8, n), dtype=torch.int32, device="cuda")
        v = torch.zeros((1 + nl, n), dtype=torch.int64, device="cuda")
        s.row_values_device(dx, dy, t, v)
        s.sync()
        return v.cpu().numpy()

    with Scanner(scan, spend, labels, max_rows=n) as fresh:
        want = values(fresh, len(labels))
    other = bytes([7]) * 32
    with Scanner(other, spend, [], max_rows=n) as s:
        values(s, 0)
        s.set_keys(scan, spend, labels)  # grows the label buffers
        assert (values(s, len(labels)) == want).all()
        s.set_keys(scan, spend, labels[:1])
        assert (values(s, 1) == want[:2]).all()


def test_multi_gpu_round_robin_host(gpu, monkeypatch):
    """The host's num_gpus > 1 path (CudaspScanLocalInit's round-robin,
    src/cudasp_extension.cu:523-529) on a one-GPU box: the test hook
    CUDASP_TF_DEVICE_MAP="0,0" gives the host two logical GPUs that both run
    on device 0.  Executor threads alternate logical GPUs 0, 1, 0, 1, each
    with its own scanner and stream, and the results equal the one-GPU run
    (as multisets) on the SQL file's queries and on 128 random rows with
    planted base and label matches repeated over several batches."""
    from cudasp_amd import cudasp_scan, release_pool
    sc = golden_io.load("sql_cases.json")
    rr = golden_io.load("random_rows.json")
    rows = [(bytes.fromhex(r["txid"]), 800000 + i,
             bytes.fromhex(r["tweak"]), r["outputs"]) for i, r in enumerate(rr["rows"])] * 40
    keys = (bytes.fromhex(rr["scan_key"]), bytes.fromhex(rr["spend_key"]),
            [bytes.fromhex(l) for l in rr["label_keys"]])

    def run_all(threads):
        outs, assign = [], []
        for q in sc["queries"]:
            outs.append(sorted(cudasp_scan(_table(sc, q), bytes.fromhex(q["scan_key"]), bytes.fromhex(q["spend_key"]),
                                           [bytes.fromhex(l) for l in q["label_keys"]], batch_size=q["batch_size"],
                                           threads=threads)))
        outs.append(sorted(cudasp_scan(rows, *keys, batch_size=1000, threads=threads, assignments=assign)))
        return outs, assign

    monkeypatch.delenv("CUDASP_TF_DEVICE_MAP", raising=False)
    one, assign1 = run_all(4)
    assert {g for g, _ in assign1} == {0}
    release_pool()
    monkeypatch.setenv("CUDASP_TF_DEVICE_MAP", "0,0")
    two, assign2 = run_all(4)
    release_pool()
    assert assign2 == [(0, 0), (1, 0), (0, 0), (1, 0)]
    assert two == one
    assert len(one[-1]) > 0
