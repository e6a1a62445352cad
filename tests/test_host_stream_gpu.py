"""GPU: the table-function host's streaming feeds (csrc/host/cudasp_host.cpp:
one persistent k_scan_stream per device, the matching rows' indices written
back into the pinned slot) beyond the default options and single query:

* two concurrent queries on one GPU with different keys, one through row
  chunks and one through Arrow columns, twice (the second round rebinds
  pooled feeds while the other query's kernel is resident), each compared
  with the C oracle's flags for its own keys (the reference is re-entrant
  per batch, src/cudasp_gpu.cu:474-484);
* output_count 2, 6, 8 and 13 (with and without label negation) on the
  streaming feed (cudasp_tf_bind_options; K hashes per row,
  src/cudasp_gpu.cu:278-282 for the index hash they extend) and 8 on
  per-slot launches, against the oracle's scan_ex;
* label keys with every output list NULL or empty (no output words in a
  slot: its device mirror still exists);
* a wait timeout (CUDASP_STREAM_TIMEOUT_MS): the query fails with an error
  instead of hanging, its feed drains and is pooled, and the next query on
  it returns the planted rows; a kernel the bounded finish gives up on is
  leaked without any wait;
* a batch made late (test hook) while ~150 small batches pass: the feed's
  ring bound harvests it before the stream runs 64 batches past it."""
import numpy as np
import pytest

import test_multi_batch_gpu as tm
from test_labels16_gpu import keys, rows_of, synth_var, torch  # noqa: F401  (fixtures + helpers)

pytestmark = pytest.mark.gpu


def _sql_keys():
    import golden_io
    q = golden_io.load("sql_cases.json")["queries"][3]
    return bytes.fromhex(q["scan_key"]), bytes.fromhex(q["spend_key"]), [bytes.fromhex(l) for l in q["label_keys"]]


def _table(torch, scan, spend, labels, first, n, kmax, every):  # noqa: F811
    """n synthetic rows (1..kmax outputs), planted values every `every` rows
    rotating over the base value and each label (oracle values), and the
    oracle's flags for them."""
    from oracle import oracle
    x, y, outs, offs, lens = synth_var(torch, first, n, kmax=kmax)
    tw = rows_of(x, y)
    o = outs.cpu().numpy()
    of = offs.cpu().numpy().view(np.uint32)
    ln = lens.cpu().numpy().view(np.uint32)
    idx = np.arange(0, n, every)
    _, ov = oracle.scan(scan, spend, labels, tw[idx], threads=16, want_values=True)
    for j, i in enumerate(idx):
        o[of[i] + ln[i] - 1] = ov[j, j % (1 + len(labels))]
    want, _ = oracle.scan(scan, spend, labels, tw, o, of, ln, threads=16)
    rows = [(int(i).to_bytes(32, "big"), 800000 + i, bytes(tw[i]), [int(v) for v in o[of[i]:of[i] + ln[i]]])
            for i in range(n)]
    return rows, sorted(np.nonzero(want)[0].tolist())


def _arrow(rows):
    import pyarrow as pa
    return pa.table({"txid": pa.array([r[0] for r in rows], pa.binary()),
                     "height": pa.array([r[1] for r in rows], pa.int32()),
                     "tweak_key": pa.array([r[2] for r in rows], pa.binary(64)),
                     "outputs": pa.array([r[3] for r in rows], pa.list_(pa.int64()))})


def test_host_concurrent_queries_different_keys(torch, keys):  # noqa: F811
    """Query A: the bench's keys with 16 labels over row chunks; query B: the
    SQL test's BIP-352 keys with its label over Arrow columns of another
    table.  They run at once on one GPU, twice; each emits exactly the
    oracle's rows for its own keys."""
    import threading
    from cudasp_amd import cudasp_scan, cudasp_scan_arrow, release_pool
    sa, pa_, la = keys
    sb, pb, lb = _sql_keys()
    rows_a, want_a = _table(torch, sa, pa_, la, 3_300_000, 12000, 15, 9)
    rows_b, want_b = _table(torch, sb, pb, lb, 7_700_000, 15000, 4, 11)
    tab_b = _arrow(rows_b)
    assert want_a and want_b
    release_pool()
    for rnd in range(2):
        out, errs = {}, []

        def run_a():
            try:
                st = {}
                got = cudasp_scan(rows_a, sa, pa_, la, batch_size=2500, threads=3, stats=st)
                out["a"] = (sorted(h - 800000 for _, h, _ in got), st)
            except Exception as e:  # noqa: BLE001 -- reported below
                errs.append(("a", repr(e)))

        def run_b():
            try:
                st = {}
                t = cudasp_scan_arrow(tab_b, sb, pb, lb, batch_size=4000, threads=4, piece_rows=3000, stats=st)
                out["b"] = (sorted(h - 800000 for h in t.column("height").to_pylist()), st)
            except Exception as e:  # noqa: BLE001
                errs.append(("b", repr(e)))

        ts = [threading.Thread(target=run_a), threading.Thread(target=run_b)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(timeout=240)
        assert not any(t.is_alive() for t in ts), "a concurrent query did not finish"
        assert not errs, errs
        assert out["a"][0] == want_a, ("a", rnd)
        assert out["b"][0] == want_b, ("b", rnd)
        for name in ("a", "b"):
            assert out[name][1]["streaming_feeds"] == 1
    release_pool()


def _variant_rows(torch, n, K, neg, labels, first):  # noqa: F811
    import variants as V  # noqa: F401
    from oracle import oracle
    from test_variants_gpu import _outputs
    b = tm.make_batch(torch, first, n)
    xs = b["tweak_x"].cpu().numpy().view(np.uint32)
    ys = b["tweak_y"].cpu().numpy().view(np.uint32)
    tw = np.ascontiguousarray(np.concatenate([xs.T, ys.T], axis=1).astype("<u4")).view(np.uint8).reshape(n, 64)
    outs, offs, lens = _outputs(tm.SCAN, tm.SPEND, labels, [{"tweak": bytes(tw[i]).hex()} for i in range(n)], K, neg,
                                False)
    want, _ = oracle.scan_ex(tm.SCAN, tm.SPEND, labels, tw, outs, offs, lens, output_count=K, label_negation=neg,
                             threads=16)
    rows = [(int(i).to_bytes(32, "big"), 800000 + i, bytes(tw[i]), [int(v) for v in outs[offs[i]:offs[i] + lens[i]]])
            for i in range(n)]
    return rows, sorted(np.nonzero(want)[0].tolist())


@pytest.mark.parametrize("K,neg,threads,batch,mode", [(2, True, 3, 2500, None), (2, True, 8, 300000, None),
                                                      (6, False, 4, 3000, None), (8, True, 3, 2500, None),
                                                      (13, False, 4, 3000, None), (8, True, 3, 2500, "launch")])
def test_host_stream_output_count(torch, monkeypatch, K, neg, threads, batch, mode):  # noqa: F811
    """output_count K with one label (and label negation) on the streaming
    feed (the host's default path; K > 6 takes the kernel's one-row pieces
    with indices in groups of 6) and, for K = 8, on per-slot launches
    (CUDASP_TF_MODE=launch); the emitted rows are the oracle's scan_ex flags."""
    from cudasp_amd import cudasp_scan, release_pool
    labels = [tm.LABEL]
    rows, want = _variant_rows(torch, 6000, K, neg, labels, 9100 + K)
    assert want
    if mode:
        monkeypatch.setenv("CUDASP_TF_MODE", mode)
    release_pool()
    st = {}
    got = cudasp_scan(rows, tm.SCAN, tm.SPEND, labels, batch_size=batch, threads=threads, output_count=K,
                      label_negation=neg, stats=st)
    assert sorted(h - 800000 for _, h, _ in got) == want
    assert st["streaming_feeds"] == (0 if mode == "launch" else 1)
    assert st["rows"] == len(rows)
    release_pool()


def test_host_stream_labels_no_output_words(torch, keys):  # noqa: F811
    """Label keys and rows whose output lists are all NULL or empty: no slot
    holds an output word, the streaming feed still publishes (its device
    mirror has a word) and the query emits nothing; then a query with
    outputs on the same pooled feed emits the oracle's rows."""
    from cudasp_amd import cudasp_scan, release_pool
    sa, pa_, la = keys
    rows, want = _table(torch, sa, pa_, la[:2], 4_400_000, 5000, 3, 13)
    empty = [(t, h, tw, None if i % 2 else []) for i, (t, h, tw, _) in enumerate(rows)]
    release_pool()
    st = {}
    assert cudasp_scan(empty, sa, pa_, la[:2], batch_size=2000, threads=3, stats=st) == []
    assert st["streaming_feeds"] == 1 and st["rows"] == len(rows)
    got = cudasp_scan(rows, sa, pa_, la[:2], batch_size=2000, threads=3)
    assert sorted(h - 800000 for _, h, _ in got) == want
    release_pool()


def _planted_arrow(torch, n, first, every=100_003):  # noqa: F811
    """n synthetic rows as an Arrow table (2 outputs per row, txid = BE row
    index, height = row index) with the true base value (C oracle) planted
    on every `every`-th row from row 17; returns (table, planted rows)."""
    import pyarrow as pa
    from oracle import oracle
    b = tm.make_batch(torch, first, n)
    xs = b["tweak_x"].cpu().numpy().view(np.uint32)
    ys = b["tweak_y"].cpu().numpy().view(np.uint32)
    tw = np.ascontiguousarray(np.concatenate([xs.T, ys.T], axis=1).astype("<u4")).view(np.uint8).reshape(n, 64)
    outs = b["outputs"][:2 * n].cpu().numpy().copy()
    planted = np.arange(17, n, every)
    _, ov = oracle.scan(tm.SCAN, tm.SPEND, [], tw[planted], threads=16, want_values=True)
    outs[2 * planted] = ov[:, 0]
    txid = np.zeros((n, 32), dtype=np.uint8)
    txid[:, 24:] = np.arange(n, dtype=">u8").view(np.uint8).reshape(n, 8)
    tab = pa.table({
        "txid": pa.FixedSizeBinaryArray.from_buffers(pa.binary(32), n, [None, pa.py_buffer(txid.tobytes())]),
        "height": pa.array(np.arange(n, dtype=np.int32)),
        "tweak_key": pa.FixedSizeBinaryArray.from_buffers(pa.binary(64), n, [None, pa.py_buffer(tw.tobytes())]),
        "outputs": pa.ListArray.from_arrays(pa.array(np.arange(0, 2 * n + 1, 2, dtype=np.int32)), pa.array(outs)),
    })
    return tab, planted


def test_host_stream_timeout_then_pooled_feed(torch, monkeypatch):  # noqa: F811
    """CUDASP_STREAM_TIMEOUT_MS=1 on a 2.4M-row Arrow query with
    batch_size 2.4M (the ramp's last slot holds 1.2M rows, ~7 ms of GPU
    work, still running when the input ends): the end-of-query wait sees no
    batch complete for 1 ms and the query fails with an error instead of
    hanging; freeing it drains the kernel with the default bound and pools
    the feed (or, if the query's own bounded finish gave up on the kernel,
    leaks it); the next query (the default timeout) emits exactly the
    planted rows."""
    from cudasp_amd import CudaspError, cudasp_scan_arrow, pool_size, release_pool
    n = 2_400_000
    tab, planted = _planted_arrow(torch, n, 123_456)
    release_pool()
    monkeypatch.setenv("CUDASP_STREAM_TIMEOUT_MS", "1")
    with pytest.raises(CudaspError) as e:
        cudasp_scan_arrow(tab, tm.SCAN, tm.SPEND, [], batch_size=n, threads=8)
    assert "without progress" in str(e.value) or "still running" in str(e.value)
    assert pool_size() <= 1  # drained and pooled, or abandoned and leaked
    monkeypatch.delenv("CUDASP_STREAM_TIMEOUT_MS")
    st = {}
    out = cudasp_scan_arrow(tab, tm.SCAN, tm.SPEND, [], batch_size=n, threads=8, stats=st)
    assert sorted(out.column("height").to_pylist()) == planted.tolist()
    assert st["streaming_feeds"] == 1
    release_pool()


def test_host_stream_abandoned_feed_is_leaked(torch, monkeypatch):  # noqa: F811
    """A kernel still running when the query's bounded finish gives up
    (CUDASP_STREAM_TIMEOUT_MS=1, one 4M-row slot: ~25 ms of GPU work, no
    ramp): the stream is abandoned, and freeing the query frees nothing the
    kernel may touch and waits for nothing -- the feed is leaked, not pooled
    (feeds_release goes straight to release_res).  The GPU then finishes the
    abandoned kernel on its own and the next query, on a new feed, emits
    exactly the planted rows."""
    from cudasp_amd import CudaspError, cudasp_scan_arrow, pool_size, release_pool
    n = 4_000_000
    tab, planted = _planted_arrow(torch, n, 7_000_001, every=250_007)
    release_pool()
    monkeypatch.setenv("CUDASP_STREAM_TIMEOUT_MS", "1")
    monkeypatch.setenv("CUDASP_TF_RAMP", "0")
    with pytest.raises(CudaspError) as e:
        cudasp_scan_arrow(tab, tm.SCAN, tm.SPEND, [], batch_size=n, threads=4)
    assert "without progress" in str(e.value) or "still running" in str(e.value)
    assert pool_size() == 0  # abandoned: leaked, never pooled
    monkeypatch.delenv("CUDASP_STREAM_TIMEOUT_MS")
    monkeypatch.delenv("CUDASP_TF_RAMP")
    out = cudasp_scan_arrow(tab, tm.SCAN, tm.SPEND, [], batch_size=300000, threads=4)
    assert sorted(out.column("height").to_pylist()) == planted.tolist()
    release_pool()


def test_host_stream_late_batch_ring_bound(torch, monkeypatch):  # noqa: F811
    """Out-of-order slot reuse cannot run the stream 64 batches past a late
    batch: 2048-row batches (~150 of them), 48 slots, no
    wave priority, and batch 3 made late by the test hook
    (CUDASP_TF_TEST_LATE_SEQ: the non-blocking checks read it as not done
    for 60 s, so the ring moves on without it).  Before the ring bound, the
    late batch was harvested more than 64 publishes later and the query
    failed (cudasp_stream_matches: not a done batch of the last 64); with it,
    the feed harvests the late slot first once the bound is reached, and the
    query emits exactly the planted rows."""
    from cudasp_amd import cudasp_scan_arrow, release_pool
    n = 300_000
    tab, planted = _planted_arrow(torch, n, 55_555, every=1_009)
    release_pool()
    monkeypatch.setenv("CUDASP_TF_STREAM_SLOTS", "48")
    monkeypatch.setenv("CUDASP_STREAM_PRIO_US", "0")
    monkeypatch.setenv("CUDASP_TF_TEST_LATE_SEQ", "3")
    monkeypatch.setenv("CUDASP_TF_TEST_LATE_MS", "60000")
    st = {}
    out = cudasp_scan_arrow(tab, tm.SCAN, tm.SPEND, [], batch_size=2048, threads=8, piece_rows=2048, stats=st)
    assert sorted(out.column("height").to_pylist()) == planted.tolist()
    assert st["streaming_feeds"] == 1 and st["launches"] > 100
    release_pool()


def test_host_e2e_eight_logical_gpus_config4():
    """The N = 8 host path rehearsed on one card at the full config-4 size
    (BASELINE.json configs[3]: 32.7M rows, 0 labels): tools/host_e2e with
    CUDASP_TF_DEVICE_MAP=0 x 8 (8 logical GPUs, threads' chunks round-robin
    over them, src/cudasp_extension.cu:523-529), 8 executor threads per
    logical GPU, one streaming feed each (CUDASP_TF_MODE=stream; each kernel
    gets 1/8 of the wave slots, GPU_MAX_HW_QUEUES=16 so every feed's stream
    has a hardware queue).  Every query emits exactly the planted rows, and
    a strided sample of 256 planted and 256 unplanted rows is recomputed by
    the C oracle (the planted values come from the GPU's values path)."""
    import json
    import os
    import subprocess
    import tempfile

    from oracle import oracle
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "tools", "host_e2e")
    env = dict(os.environ, CUDASP_TF_DEVICE_MAP=",".join(["0"] * 8), CUDASP_TF_MODE="stream",
               GPU_MAX_HW_QUEUES="16")
    sample = os.path.join(tempfile.mkdtemp(), "sample.json")
    cmd = [exe, "--rows", "32700000", "--threads", "64", "--batch", "300000", "--labels", "0", "--input", "rows",
           "--reps", "1", "--outputs", "2", "--plant-sample", sample]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=280, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-2000:])
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["logical_gpus"] == 8
    assert res["feeds"] == 8 and res["streaming_feeds"] == 8
    assert res["emitted_equal_planted"] is True
    assert res["matches"] == res["planted"] == 32700
    chk = oracle.check_planted_sample(json.load(open(sample)), threads=16)
    assert chk["rows"] == 512 and chk["planted"] == 256 and chk["equal"] == chk["rows"], chk
    print("8 logical GPUs, 64 threads, 32.7M rows: %.1f M tx/s on one card" % (res["tx_per_s"] / 1e6))


@pytest.mark.parametrize("labels,threads,batch,rows,outs", [(2, 16, 1, 65536, ["--outputs", "2"]),
                                                             (0, 1, 2048, 65536, ["--outputs", "2"]),
                                                             (1, 3, 2048, 300001, ["--outputs-max", "15"]),
                                                             (0, 1, 2048, 300001, ["--outputs", "8"]),
                                                             (1, 4, 2048, 65536, ["--outputs", "2", "--output-count", "8"])])
def test_host_stream_slot_reuse_reads_fresh_rows(labels, threads, batch, rows, outs):
    """A streaming feed with 4 slots (CUDASP_TF_STREAM_SLOTS=4) and 2048-row
    batches: every slot -- its pinned rows and its device mirror of the
    outputs -- is rewritten for a newer batch while the persistent kernel
    runs, a few batches after the kernel last read it.  Each iteration's reads
    follow a system-scope acquire and the mirror is written through, so no
    row is scanned with a stale tweak or compared with a stale outputs list
    (without the acquire 8-25% of the planted matches were lost, without the
    write-through 1-3 per query; profiles/r05_stream_acquire.txt).  The last
    case streams output_count 8 through the WIDE instance, which reads a
    piece's mirrors in the iteration that wrote them (after a vmcnt wait and an
    agent-scope acquire).  Every
    query emits exactly the planted rows; the oracle recomputes the run's
    sample."""
    import json
    import os
    import subprocess
    import tempfile

    import bench
    from oracle import oracle
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "tools", "host_e2e")
    d = tempfile.mkdtemp()
    sample, lf = os.path.join(d, "sample.json"), os.path.join(d, "labels.bin")
    env = dict(os.environ, CUDASP_TF_DEVICE_MAP="0", CUDASP_TF_STREAM_SLOTS="4")
    env.pop("CUDASP_TF_MODE", None)
    cmd = [exe, "--rows", str(rows), "--threads", str(threads), "--batch", str(batch), "--labels", str(labels),
           "--input", "rows", "--reps", "3", "--plant-sample", sample] + outs
    if labels:
        with open(lf, "wb") as f:
            f.write(b"".join(bench.label_keys(labels)))
        cmd += ["--labels-file", lf]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=100, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-2000:])
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["streaming_feeds"] == 1 and res["launches"] >= rows // 2048
    assert res["emitted_equal_planted"] is True and res["matches"] == res["planted"]
    chk = oracle.check_planted_sample(json.load(open(sample)), threads=8)
    assert chk["equal"] == chk["rows"] > 0, chk
