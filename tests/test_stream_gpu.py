"""GPU: the streaming scan (cudasp_stream_*: ONE persistent k_scan_stream
kernel scans batches as they are published, reading them from coherent pinned
host memory and writing their flags back there) gives the per-batch path's
flags -- ragged batch sizes, 0 / 2 / 16 labels (the label compares read the
device mirror of each row's outputs), 1..15 outputs per row, a ring that
wraps, reuse after finish, a slow publisher and an idle host (the kernel
leaves and is relaunched), exceptional label sums in one thread's piece, and the C
oracle."""
import os
import time

import numpy as np
import pytest

import test_multi_batch_gpu as tm
from test_multi_batch_gpu import torch  # noqa: F401  (fixture)

pytestmark = pytest.mark.gpu

# a kernel with nothing to do leaves after this many milliseconds (the
# default; the host's next publish or wait relaunches it)
os.environ.setdefault("CUDASP_STREAM_IDLE_MS", "20")

SCAN, SPEND, LABEL = tm.SCAN, tm.SPEND, tm.LABEL


def host_rows(b):
    """A device batch's tweak columns as the table's 64-byte row blobs."""
    xs = b["tweak_x"].cpu().numpy().view(np.uint32)
    ys = b["tweak_y"].cpu().numpy().view(np.uint32)
    n = b["n"]
    return np.ascontiguousarray(np.concatenate([xs.T, ys.T], axis=1).astype("<u4")).view(np.uint8).reshape(n, 64)


def staged(b, label_count):
    from cudasp_amd import StreamBatch
    n = b["n"]
    return StreamBatch(host_rows(b), b["outputs"].cpu().numpy(), b["offsets"][:n].cpu().numpy().view(np.uint32),
                       b["lengths"][:n].cpu().numpy().view(np.uint32), label_count=label_count)


def run_stream(batches, labels, rounds=1, max_in_flight=None):
    """Publish every batch into one stream (`rounds` queries on the same
    stream), waiting for the oldest when max_in_flight are out; returns the
    last round's flags per batch and the stream's stats.  Every batch's
    compacted matches (match_rows, cudasp_stream_matches) are its flagged
    rows."""
    from cudasp_amd import Scanner, ScanStream
    stage = [staged(b, len(labels)) for b in batches]
    with Scanner(SCAN, SPEND, labels, max_rows=1000) as s, ScanStream(s) as st:
        for _ in range(rounds):
            for sb in stage:
                sb.reset()
            seqs = []
            for sb in stage:
                if max_in_flight and len(seqs) >= max_in_flight:
                    st.wait(seqs[-max_in_flight])
                seqs.append(sb.publish(st))
            st.close_input()
            for q in seqs:
                st.wait(q)
            assert all(st.query(q) for q in seqs)
            for sb in stage[-64:]:  # match counts of the last 64 batches stay readable
                assert (sb.matches(st) == np.nonzero(sb.result())[0]).all()
            st.finish()
        stats = st.stats()
    return [sb.result() for sb in stage], stats


def flags_equal(got, want):
    assert len(got) == len(want)
    for i, (g, (w, _, _)) in enumerate(zip(got, want)):
        assert (g == w).all(), "batch %d: %d rows differ" % (i, int((g != w).sum()))


SIZES = [3001, 64, 1, 129, 70000, 65, 2047, 300000]


@pytest.mark.parametrize("nlabels", [0, 2])
def test_stream_equals_per_batch(torch, nlabels):
    labels = [LABEL, SPEND][:nlabels]
    batches = [tm.make_batch(torch, 1000 + 300000 * i, n) for i, n in enumerate(SIZES)]
    tm.plant(torch, batches, labels)
    want = tm.run_per_batch(torch, batches, labels)
    assert sum(c for _, _, c in want) > 0
    got, stats = run_stream(batches, labels, rounds=2)
    flags_equal(got, want)
    assert stats["launches"] >= 2  # one kernel per query at least


def test_stream_16_labels_variable_outputs(torch):
    """Config-5 shape: 16 labels, 1..15 outputs per row, planted values over
    every label index; matches the per-batch path and the C oracle."""
    from oracle import oracle
    labels = tm.labels16()
    batches = [tm.make_batch(torch, 3 + 40000 * i, n, kmax=15) for i, n in enumerate([5000, 333, 4096, 1])]
    tm.plant(torch, batches, labels, every=7)
    want = tm.run_per_batch(torch, batches, labels)
    assert sum(c for _, _, c in want) > 1000
    got, _ = run_stream(batches, labels)
    flags_equal(got, want)
    b = batches[1]
    n = b["n"]
    ref, _ = oracle.scan(SCAN, SPEND, labels, host_rows(b), b["outputs"].cpu().numpy(),
                         b["offsets"][:n].cpu().numpy().view(np.uint32),
                         b["lengths"][:n].cpu().numpy().view(np.uint32), threads=16)
    assert (got[1] == ref).all()


def test_stream_ring_wraps(torch):
    """150 batches of 1..700 rows through the 64-entry descriptor ring with
    at most 40 in flight, and then all of a second query: flags equal the
    per-batch path's over the whole table."""
    rng = np.random.default_rng(150)
    sizes = [int(x) for x in rng.integers(1, 701, 150)]
    labels = [LABEL]
    batches = [tm.make_batch(torch, 77 + 1000 * i, n) for i, n in enumerate(sizes)]
    tm.plant(torch, batches, labels, every=5)
    want = tm.run_per_batch(torch, batches, labels)
    got, _ = run_stream(batches, labels, rounds=2, max_in_flight=40)
    flags_equal(got, want)


def test_stream_reused_buffers(torch):
    """Four StreamBatch buffers carry 48 different batches in one query, each
    refilled (rows, outputs, offsets, lengths and the same device mirror)
    as soon as its previous batch is done -- a host's slot ring.  The kernel
    reads every refill fresh: flags equal the per-batch path's for every
    batch.  (Paced by Python, this does not reproduce the stale reads of
    profiles/r05_stream_acquire.txt -- it passes on the build without the
    acquire too; test_host_stream_slot_reuse_reads_fresh_rows does.)"""
    from cudasp_amd import Scanner, ScanStream
    rng = np.random.default_rng(48)
    sizes = [int(x) for x in rng.integers(500, 2049, 48)]
    labels = [LABEL]
    batches = [tm.make_batch(torch, 5 + 2048 * i, n, kmax=8) for i, n in enumerate(sizes)]
    tm.plant(torch, batches, labels, every=3)
    want = tm.run_per_batch(torch, batches, labels)
    assert sum(c for _, _, c in want) > 0
    ring = [staged(tm.make_batch(torch, 10**9 + i, 2048, kmax=15), len(labels)) for i in range(4)]
    got = [None] * len(batches)
    with Scanner(SCAN, SPEND, labels, max_rows=1000) as s, ScanStream(s) as st:
        held = [None] * len(ring)  # batch index each buffer carries
        for i, b in enumerate(batches):
            k = i % len(ring)
            sb = ring[k]
            if held[k] is not None:
                st.wait(sb.seq)
                got[held[k]] = sb.result()
            n = b["n"]
            sb.refill(host_rows(b), b["outputs"].cpu().numpy(), b["offsets"][:n].cpu().numpy().view(np.uint32),
                      b["lengths"][:n].cpu().numpy().view(np.uint32))
            sb.publish(st)
            held[k] = i
        st.close_input()
        for k, sb in enumerate(ring):
            st.wait(sb.seq)
            got[held[k]] = sb.result()
        st.finish()
    flags_equal(got, want)


def test_stream_concurrent_publishers_16_labels(torch):
    """Three publisher threads into one stream, 2500-row batches, 16 labels,
    1..15 outputs per row (the host's feed shape whose DMA-staged variant
    stalled in round 4; batches are read in place): every thread publishes
    its batches and waits for them under a 30 s no-progress deadline, and
    the flags equal the per-batch path's."""
    import threading

    from cudasp_amd import Scanner, ScanStream
    labels = tm.labels16()
    batches = [tm.make_batch(torch, 200000 + 2500 * i, 2500, kmax=15) for i in range(12)]
    tm.plant(torch, batches, labels, every=13)
    want = tm.run_per_batch(torch, batches, labels)
    stage = [staged(b, len(labels)) for b in batches]
    errors = []
    with Scanner(SCAN, SPEND, labels, max_rows=1000) as s, ScanStream(s) as st:
        st.set_timeout(30000)
        for _ in range(2):
            for sb in stage:
                sb.reset()

            def publisher(k):
                try:
                    mine = [sb.publish(st) for sb in stage[k::3]]
                    for q in mine:
                        st.wait(q)
                except Exception as e:  # noqa: BLE001 (reported below)
                    errors.append(e)

            th = [threading.Thread(target=publisher, args=(k,)) for k in range(3)]
            for t in th:
                t.start()
            for t in th:
                t.join(timeout=60)
            assert not any(t.is_alive() for t in th), "a publisher thread did not finish"
            assert not errors, errors
            st.finish()
    flags_equal([sb.result() for sb in stage], want)
    assert sum(c for _, _, c in want) > 0


def test_stream_slow_publisher(torch):
    """Batches published 50 ms apart, longer than the 20 ms idle time: the
    kernel leaves after each batch (the GPU is not held while the host is
    slow) and the next publish relaunches it; the results are the per-batch
    path's."""
    from cudasp_amd import Scanner, ScanStream
    labels = [LABEL]
    batches = [tm.make_batch(torch, 5000 + 9000 * i, n) for i, n in enumerate([4000, 700, 8000])]
    tm.plant(torch, batches, labels, every=9)
    want = tm.run_per_batch(torch, batches, labels)
    stage = [staged(b, 1) for b in batches]
    with Scanner(SCAN, SPEND, labels, max_rows=1000) as s, ScanStream(s) as st:
        for sb in stage:
            q = sb.publish(st)
            st.wait(q)
            time.sleep(0.05)
        st.finish()
        c = st.counters()  # the finished query's, summed over its launches
        launches = st.stats()["launches"]
    assert launches == 3
    assert c["idle_exits"] >= 2
    assert c["wave_rows"] == sum((b["n"] + 63) // 64 for b in batches)
    flags_equal([sb.result() for sb in stage], want)


def test_stream_publish_around_idle_exit(torch):
    """Publishes that land while the kernel is leaving: 40 batches, each after
    a pause drawn around the 20 ms idle time (0, 17..23 ms), some waited for
    and some not -- the poller's idle exit, the host's relaunch and the
    claim counter's reset to pub_wr race on every batch.  Every batch's
    flags are the per-batch path's, and the query's counters account for
    every wave-row exactly once."""
    from cudasp_amd import Scanner, ScanStream
    rng = np.random.default_rng(4020)
    labels = [LABEL]
    sizes = [int(x) for x in rng.integers(1, 3000, 40)]
    batches = [tm.make_batch(torch, 91000 + 4000 * i, n) for i, n in enumerate(sizes)]
    tm.plant(torch, batches, labels, every=11)
    want = tm.run_per_batch(torch, batches, labels)
    stage = [staged(b, 1) for b in batches]
    pauses = rng.choice([0.0, 0.017, 0.019, 0.020, 0.021, 0.023], size=len(stage))
    with Scanner(SCAN, SPEND, labels, max_rows=1000) as s, ScanStream(s) as st:
        seqs = []
        for i, sb in enumerate(stage):
            time.sleep(float(pauses[i]))
            seqs.append(sb.publish(st))
            if i % 3 == 0:
                st.wait(seqs[-1])
        st.close_input()
        for q in seqs:
            st.wait(q)
        st.finish()
        c = st.counters()
        launches = st.stats()["launches"]
    assert c["wave_rows"] == sum((n + 63) // 64 for n in sizes)
    assert launches >= 2  # some pauses outlasted the idle time
    flags_equal([sb.result() for sb in stage], want)


def test_stream_idle_kernel_releases_gpu(torch):
    """While a stream is open but the host publishes nothing, the kernel
    leaves after the idle time, so other work on the GPU runs (a kernel that
    held every wave slot until the stream closed would stall it); the next
    publish relaunches it and a later query on the stream is unaffected."""
    from cudasp_amd import Scanner, ScanStream
    b = tm.make_batch(torch, 99, 3000)
    tm.plant(torch, [b], [], every=50)
    want = tm.run_per_batch(torch, [b], [])
    sb = staged(b, 0)
    with Scanner(SCAN, SPEND, [], max_rows=1000) as s, ScanStream(s) as st:
        st.wait(sb.publish(st))
        time.sleep(0.1)
        x = torch.ones(1 << 20, device="cuda")
        t = time.perf_counter()
        y = (x * 3).sum()
        torch.cuda.synchronize()
        assert float(y) == 3 * (1 << 20)
        assert time.perf_counter() - t < 5
        sb.flags.array[:] = 0xEE
        st.wait(sb.publish(st))
        st.finish()
        assert st.stats()["launches"] == 2
        flags_equal([sb.result()], want)
        sb.flags.array[:] = 0xEE
        st.wait(sb.publish(st))
        st.finish()
    flags_equal([sb.result()], want)


def test_stream_exceptional_label_sums(torch):
    """Label keys that make label sums exceptional inside one thread's piece
    (test_multi_exceptional_label_sums' construction): F + L = 2F matches, a
    sum at infinity never does; flags equal the oracle's."""
    import variants as V
    from oracle import oracle
    n = 64 * 6 * 2 + 17
    b = tm.make_batch(torch, 31337, n)
    tw = host_rows(b)
    ra, rb, rc = 5, 5 + 64, 5 + 128
    F = [V.row(SCAN, SPEND, [], bytes(tw[i]))[0][0][0] for i in (ra, rb, rc)]
    labels = [V.point_blob(F[0]), LABEL, V.point_blob(V.neg(F[1])), V.point_blob(F[2])]
    _, vals = oracle.scan(SCAN, SPEND, labels, tw, want_values=True)
    outs = b["outputs"].cpu().numpy()
    offs = b["offsets"][:n].cpu().numpy().view(np.uint32)
    lens = b["lengths"][:n].cpu().numpy().view(np.uint32)
    for i in range(n):
        if i in (ra, rb, rc):
            continue
        if i % 11 == 0:
            outs[offs[i]] = vals[i, 0]
        elif i % 9 == 0:
            outs[offs[i] + 1] = vals[i, 2]
    outs[offs[ra]] = vals[ra, 1]
    outs[offs[rb]] = oracle.LABEL_INFINITY
    outs[offs[rb] + 1] = 0
    outs[offs[rc] + 1] = vals[rc, 4]
    b["outputs"] = torch.from_numpy(outs).cuda()
    want, _ = oracle.scan(SCAN, SPEND, labels, tw, outs, offs, lens, threads=16)
    assert want[ra] == 1 and want[rb] == 0 and want[rc] == 1
    got, _ = run_stream([b], labels)
    assert (got[0] == want).all()


def test_stream_rejects_bad_use(torch):
    from cudasp_amd import CudaspError, HostBuffer, Scanner, ScanStream, StreamBatch
    b = tm.make_batch(torch, 1, 100)
    with Scanner(SCAN, SPEND, [LABEL], max_rows=100) as s:
        with ScanStream(s) as st:
            sb = staged(b, 1)
            with pytest.raises(CudaspError):  # no outputs mirror
                st.publish(sb.rows, sb.outputs, sb.offsets, sb.lengths, sb.n, sb.flags, None)
            with pytest.raises(CudaspError):  # empty batch
                st.publish(sb.rows, sb.outputs, sb.offsets, sb.lengths, 0, sb.flags, sb.mirror)
            with pytest.raises(CudaspError):  # neither flags nor match rows
                st.publish(sb.rows, sb.outputs, sb.offsets, sb.lengths, sb.n, None, sb.mirror)
            # host buffers outside cudasp_host_alloc (pageable memory): refused,
            # the kernel's uncached reads and system-scope stores need coherent memory
            pageable = np.zeros(100 * 64, dtype=np.uint8)
            with pytest.raises(CudaspError):
                st.publish(pageable.ctypes.data, sb.outputs, sb.offsets, sb.lengths, sb.n, sb.flags, sb.mirror)
            part = HostBuffer(64 * 50)  # coherent, but smaller than the batch
            with pytest.raises(CudaspError):
                st.publish(part, sb.outputs, sb.offsets, sb.lengths, sb.n, sb.flags, sb.mirror)
            part.close()
            # still usable after the refusals
            q = sb.publish(st)
            st.wait(q)
            st.finish()
        s.set_fixed_base_bits(7)  # the LDS-staged width: stage B of the stream reads an HBM table
        with pytest.raises(CudaspError):
            ScanStream(s)
    assert StreamBatch is not None


def _variant_case(torch, n, K, neg, full_x, labels, first):
    """n synthetic rows with a decoy and, on 4 of 5 rows, one planted
    candidate chosen round-robin over every (output index, value column)
    of the variant (test_variants_gpu's construction); the oracle's flags."""
    from oracle import oracle
    from test_variants_gpu import _outputs
    b = tm.make_batch(torch, first, n)
    tw = host_rows(b)
    rows = [{"tweak": bytes(tw[i]).hex()} for i in range(n)]
    outs, offs, lens = _outputs(SCAN, SPEND, labels, rows, K, neg, full_x)
    want, _ = oracle.scan_ex(SCAN, SPEND, labels, tw, outs, offs, lens, output_count=K, label_negation=neg,
                             full_x=full_x, threads=16)
    return tw, outs, offs, lens, want


@pytest.mark.parametrize("K,neg,full_x", [(2, True, False), (2, False, False), (3, False, True), (6, True, False),
                                          (7, False, False), (8, True, False), (13, False, True), (64, True, False)])
def test_stream_variants(torch, K, neg, full_x):
    """output_count K > 1 (K hashes and fixed-base points per row: K x rows
    per piece <= 6 in the pipelined schedule; K > 6 one row per piece, its
    indices in groups of 6 with their own inversions, 13 = 6 + 6 + 1), label
    negation and full-x compares through the streaming kernel: flags and
    compacted matches equal the C oracle's scan_ex over ragged batches in
    one stream (the reference has none of the variants: parity unpinned
    against it, pinned to tests/variants.py)."""
    from cudasp_amd import Scanner, ScanStream, StreamBatch
    labels = [LABEL]
    n = 700 if full_x or K > 16 else 2200
    tw, outs, offs, lens, want = _variant_case(torch, n, K, neg, full_x, labels, 4242 + K)
    assert 0 < int(want.sum()) < n
    cuts = [0, 1, 65, n // 2, n]
    ow = 32 if full_x else 1
    stage = []
    for a, z in zip(cuts[:-1], cuts[1:]):
        o0 = int(offs[a])
        o1 = int(offs[z - 1] + lens[z - 1])
        sub = outs[o0:o1]
        stage.append(StreamBatch(tw[a:z], sub, offs[a:z] - o0, lens[a:z], label_count=1, full_x=full_x,
                                 want_flags=(K != 3)))
    del ow
    with Scanner(SCAN, SPEND, labels, max_rows=1000) as s:
        s.set_options(output_count=K, label_negation=neg, full_x=full_x)
        with ScanStream(s) as st:
            seqs = [sb.publish(st) for sb in stage]
            st.close_input()
            for q in seqs:
                st.wait(q)
            got_rows = np.concatenate([sb.matches(st) + a for sb, a in zip(stage, cuts[:-1])])
            if K != 3:
                got_flags = np.concatenate([sb.result() for sb in stage])
                assert (got_flags == want).all()
            st.finish()
    assert (got_rows == np.nonzero(want)[0]).all()


def test_stream_timeout_then_recovers(torch):
    """A wait that sees no batch complete for the stream's timeout fails with
    an error instead of hanging (cudasp_stream_set_timeout; a 2.4M-row batch
    takes > 10 ms); finish with the normal timeout then lets the batch
    complete and resets the stream, and the next query on it returns the
    per-batch path's flags."""
    from cudasp_amd import CudaspError, Scanner, ScanStream
    b = tm.make_batch(torch, 777, 2_400_000)
    tm.plant(torch, [b], [], every=100_003)
    sb = staged(b, 0)
    with Scanner(SCAN, SPEND, [], max_rows=1000) as s, ScanStream(s) as st:
        st.set_timeout(1)
        q = sb.publish(st)
        with pytest.raises(CudaspError) as e:
            st.wait(q)
        assert "without progress" in str(e.value)
        st.set_timeout(60000)
        st.finish()
        assert not st.abandoned()
        first = sb.result()
        sb.reset()
        q = sb.publish(st)
        st.wait(q)
        st.finish()
        again = sb.result()
    want = tm.run_per_batch(torch, [b], [])
    assert (again == want[0][0]).all()
    assert (first == want[0][0]).all()  # the timed-out wait's batch completed all the same
