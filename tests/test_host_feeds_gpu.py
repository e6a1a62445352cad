"""GPU: the table-function host's device feeds at the config-5 shape
(BASELINE.json configs[4]: 16 label keys, 1..15 outputs per row) against the
C oracle, through the C++ host (include/cudasp_host.h) exactly as DuckDB's
executor drives it.

The host batches rows per device, not per thread (csrc/host/cudasp_host.cpp:
all executor threads fill one ring of batch slots per GPU; a slot that holds
>= batch_size rows is launched by the last thread copying into it, up to 3
launches in flight per device at the default 4 hardware queues).  These tests run several executor threads
over enough rows for many slots, with several launches in flight and the
ring wrapping, and compare the emitted multiset of rows with the oracle's
flags: row chunks and Arrow columns, one GPU and four logical GPUs on one
card (CUDASP_TF_DEVICE_MAP="0,0,0,0", fewer threads than GPUs), the
label loop of src/cudasp_gpu.cu:153-172 and the per-thread batch plumbing of
src/cudasp_extension.cu:188-223."""
import os
import subprocess
import sys

import numpy as np
import pytest

from test_labels16_gpu import keys, rows_of, synth_var, torch  # noqa: F401  (fixtures + helpers)

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N_ROWS = 24000


@pytest.fixture(scope="module")
def table16(torch, keys):  # noqa: F811
    """24000 synthetic rows with 1..15 outputs, a planted value every 7th row
    rotating over the base output and all 16 labels (in the list's last
    slot), and the oracle's flags for them."""
    from oracle import oracle
    scan, spend, labels = keys
    x, y, outs, offs, lens = synth_var(torch, 5_550_000, N_ROWS)
    tw = rows_of(x, y)
    _, ov = oracle.scan(scan, spend, labels, tw, threads=16, want_values=True)
    o = outs.cpu().numpy()
    of = offs.cpu().numpy().view(np.uint32)
    ln = lens.cpu().numpy().view(np.uint32)
    planted_cols = set()
    for i in range(0, N_ROWS, 7):
        col = (i // 7) % 17
        o[of[i] + ln[i] - 1] = ov[i, col]
        planted_cols.add(col)
    assert planted_cols == set(range(17))
    want, _ = oracle.scan(scan, spend, labels, tw, o, of, ln, threads=16)
    assert int(want.sum()) >= N_ROWS // 7
    rows = []
    for i in range(N_ROWS):
        lst = [int(v) for v in o[of[i]:of[i] + ln[i]]]
        rows.append((i.to_bytes(32, "big"), 800000 + i, bytes(tw[i]), lst))
    expected = sorted(np.nonzero(want)[0].tolist())
    return rows, expected


def _heights(out):
    return sorted(h - 800000 for _, h, _ in out)


def _check_rows(out, rows):
    for txid, h, tweak in out:
        r = rows[h - 800000]
        assert (txid, tweak) == (r[0], r[2])


@pytest.mark.parametrize("threads,batch", [(3, 2500), (8, 4000), (5, 300000)])
def test_host_feed_16_labels_rows(table16, keys, threads, batch):  # noqa: F811
    """Row chunks: several threads, batch sizes giving ~10 launches with the
    ring wrapping (2500 rows: two 2048-row chunks per slot), and one batch
    larger than the table (the ramp's first slot, then the final partial
    slot)."""
    from cudasp_amd import cudasp_scan, release_pool
    rows, expected = table16
    scan, spend, labels = keys
    stats = {}
    out = cudasp_scan(rows, scan, spend, labels, batch_size=batch, threads=threads, stats=stats)
    assert _heights(out) == expected
    _check_rows(out, rows)
    assert stats["rows"] == len(rows)
    assert stats["feeds"] == 1
    if batch < len(rows):
        assert stats["launches"] >= 3
    else:
        # the streaming feed's ramp (batch_size / 32, / 16, ...) closes its
        # first slots early: 9375 rows, then the final partial slot
        assert stats["launches"] <= 2
    assert stats["streams_per_feed"] < stats["hw_queues"]  # one queue is the null stream's
    release_pool()


def test_host_feed_16_labels_arrow(table16, keys):  # noqa: F811
    """Arrow columns (cudasp_tf_function_columns) of the same rows: same emitted rows."""
    import pyarrow as pa
    from cudasp_amd import cudasp_scan_arrow
    rows, expected = table16
    scan, spend, labels = keys
    t = pa.table({"txid": pa.array([r[0] for r in rows], pa.binary()),
                  "height": pa.array([r[1] for r in rows], pa.int32()),
                  "tweak_key": pa.array([r[2] for r in rows], pa.binary(64)),
                  "outputs": pa.array([r[3] for r in rows], pa.list_(pa.int64()))})
    stats = {}
    out = cudasp_scan_arrow(t, scan, spend, labels, batch_size=3000, threads=4, piece_rows=5000, stats=stats)
    got = sorted(h - 800000 for h in out.column("height").to_pylist())
    assert got == expected
    assert stats["rows"] == len(rows) and stats["launches"] >= 3


def test_host_feed_four_logical_gpus(table16, keys, monkeypatch):  # noqa: F811
    """Four logical GPUs on one card (CUDASP_TF_DEVICE_MAP="0,0,0,0"), each
    with its own feed, fed by two executor threads (fewer threads than GPUs:
    a thread's chunks go round-robin over all of them): the emitted multiset
    equals the one-GPU run's."""
    from cudasp_amd import cudasp_scan, release_pool
    rows, expected = table16
    scan, spend, labels = keys
    monkeypatch.delenv("CUDASP_TF_DEVICE_MAP", raising=False)
    one = cudasp_scan(rows, scan, spend, labels, batch_size=2500, threads=2)
    release_pool()
    monkeypatch.setenv("CUDASP_TF_DEVICE_MAP", "0,0,0,0")
    # 4 feeds x 2 streams on one device: more streams than hardware queues,
    # which the host reports (stats) and warns about; results do not depend on it
    monkeypatch.setenv("CUDASP_TF_STREAMS", "2")
    stats, assign = {}, []
    four = cudasp_scan(rows, scan, spend, labels, batch_size=2500, threads=2, stats=stats, assignments=assign)
    release_pool()
    assert assign == [(0, 0), (1, 0)]
    assert stats["feeds"] == 4
    assert stats["max_streams_per_device"] == 8
    assert sorted(one) == sorted(four)
    assert _heights(four) == expected


def test_host_small_table_many_threads(table16, keys):  # noqa: F811
    """A table far smaller than threads x batch_size (the 1M-row config at a
    smaller scale): 16 threads, default batch_size -- every row reaches the
    GPU through the final partial slot of the one feed."""
    from cudasp_amd import cudasp_scan
    rows, expected = table16
    scan, spend, labels = keys
    sub = rows[:5000]
    stats = {}
    out = cudasp_scan(sub, scan, spend, labels, threads=16, stats=stats)
    assert _heights(out) == [e for e in expected if e < 5000]
    assert stats["launches"] == 1 and stats["rows"] == 5000


def test_host_e2e_tool_config5_shape(torch, keys, tmp_path):  # noqa: F811
    """tools/host_e2e (the bench's PCIe-inclusive leg) at the config-5 shape:
    16 distinct label keys (bench.label_keys), 1..15 outputs per row, 8
    executor threads, row chunks and Arrow columns: every query emits exactly
    the planted rows (base values on rows 0 mod 1000, label j = (g / 1000)
    mod 16 on rows 1 mod 1000: all 16 label indices), also for a query started
    right after a busy kernel (--warm-reps).  A strided sample of planted and
    unplanted rows, with every label column, is recomputed by the C oracle."""
    import json

    from oracle import oracle
    exe = os.path.join(ROOT, "tools", "host_e2e")
    if not os.path.exists(exe):
        pytest.fail("tools/host_e2e not built (make -C duckdb-cudasp-extension_amd)")
    lf = tmp_path / "labels.bin"
    lf.write_bytes(b"".join(keys[2]))
    for mode in ("rows", "columns"):
        cmd = [exe, "--rows", "700000", "--threads", "8", "--batch", "300000", "--labels", "16",
               "--labels-file", str(lf), "--outputs-max", "15", "--input", mode, "--warm-reps", "1",
               "--plant-sample", str(tmp_path / "sample.json")]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, (mode, r.stdout[-2000:], r.stderr[-2000:])
        res = json.loads(r.stdout.strip().splitlines()[-1])
        assert res["emitted_equal_planted"] is True
        assert res["matches"] == res["planted"] == 1400
        assert res["label_indices_planted"] == 16
        assert res["launches"] >= 3
        # one more query right after a busy kernel on the GPU (bench's e2e_warm_tx_s); exit 0 covers its rows
        assert res["warm_reps"] == 1 and res["warm_tx_per_s"] > 0
        chk = oracle.check_planted_sample(json.load(open(tmp_path / "sample.json")), threads=16)
        assert chk["equal"] == chk["rows"] == 512 and chk["label_columns"] == list(range(1, 17)), chk


def test_host_error_mid_query_then_pool_reuse(table16, keys):  # noqa: F811
    """A 63-byte tweak in a late chunk of a 3-thread query: the query fails
    with an error (the reference reads 64 bytes regardless,
    src/cudasp_extension.cu:59-75) while the other threads' batches are in
    flight; freeing the global state drains them and parks the feed, and the
    next query on the pooled resources emits exactly the oracle's rows."""
    from cudasp_amd import CudaspError, cudasp_scan, pool_size
    rows, expected = table16
    scan, spend, labels = keys
    bad = list(rows[:12000])
    t = bad[9000]
    bad[9000] = (t[0], t[1], t[2][:63], t[3])
    with pytest.raises(CudaspError):
        cudasp_scan(bad, scan, spend, labels, batch_size=2500, threads=3)
    assert pool_size() > 0
    out = cudasp_scan(rows, scan, spend, labels, batch_size=2500, threads=3)
    assert _heights(out) == expected


@pytest.mark.parametrize("threads,batch", [(3, 2500), (8, 300000)])
def test_host_streaming_feed_16_labels(table16, keys, threads, batch, monkeypatch):  # noqa: F811
    """Streaming feeds (the host's default, CUDASP_TF_MODE=stream: each
    closed slot is published to the feed's one persistent k_scan_stream
    kernel, which reads it from pinned host memory in place): the emitted
    rows are the oracle's, through the final partial slot alone and through
    many slots; the per-slot launches (CUDASP_TF_MODE=launch) give the same
    result."""
    from cudasp_amd import cudasp_scan, release_pool
    rows, expected = table16
    scan, spend, labels = keys
    monkeypatch.setenv("CUDASP_TF_MODE", "stream")
    release_pool()
    stats = {}
    out = cudasp_scan(rows, scan, spend, labels, batch_size=batch, threads=threads, stats=stats)
    assert stats["streaming_feeds"] == 1
    assert _heights(out) == expected
    _check_rows(out, rows)
    assert stats["rows"] == len(rows)
    monkeypatch.setenv("CUDASP_TF_MODE", "launch")
    stats = {}
    out = cudasp_scan(rows, scan, spend, labels, batch_size=batch, threads=threads, stats=stats)
    assert stats["streaming_feeds"] == 0
    assert _heights(out) == expected
    release_pool()


def test_host_concurrent_queries_one_gpu(table16, keys):  # noqa: F811
    """Two queries at once on one GPU over the same table and keys, each
    with its own executor threads and batch size (two DuckDB connections in
    one process): each query's streaming feed runs its own kernel, and a
    kernel holds the GPU only while its query has work (it leaves after
    CUDASP_STREAM_IDLE_MS idle) -- both finish with the oracle's rows.
    Different keys, label sets and input paths at once:
    test_host_stream_gpu.py::test_host_concurrent_queries_different_keys."""
    import threading
    from cudasp_amd import cudasp_scan, release_pool
    rows, expected = table16
    scan, spend, labels = keys
    out, errs = {}, []

    def run(name, batch, threads):
        try:
            st = {}
            out[name] = (cudasp_scan(rows, scan, spend, labels, batch_size=batch, threads=threads, stats=st), st)
        except Exception as e:  # noqa: BLE001 -- reported below
            errs.append((name, repr(e)))

    ts = [threading.Thread(target=run, args=("a", 2500, 3)), threading.Thread(target=run, args=("b", 4000, 4))]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=240)
    assert not any(t.is_alive() for t in ts), "a concurrent query did not finish"
    assert not errs, errs
    for name in ("a", "b"):
        got, st = out[name]
        assert _heights(got) == expected, name
        assert st["streaming_feeds"] == 1
    release_pool()
