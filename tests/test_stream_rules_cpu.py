"""CPU replay of the streaming scan's scheduling rules
(duckdb-cudasp-extension_amd/csrc/scan_stream.hpp, k_scan_stream in
scan_kernels.hip): the ticket size rule, and the descriptor-ring lookup a wave
makes for each of its wave-rows -- a walk forward from its hint, started no
earlier than pub - STREAM_RING, skipping entries that hold another batch.

The replay drives the host's publish rule (batch X only once X - STREAM_RING
is done) with batches completing out of order, and checks that every lookup
of a not-yet-done wave-row finds its batch within three passes of the ring,
including a wave whose first hint is 0 after the ring has wrapped many times
(the case a walk from the hint alone missed) and a stale `pub` one poller
pass behind."""
import random

STREAM_RING = 64


def stream_piece_rows(rem, claimed, mine, rmax):
    if mine == 0 or claimed == 0:
        return 1
    return max(1, min(rmax, rem * mine // claimed))


def batch_of(ring, pub, hint, w):
    """stream_batch_of: ring[e] = (seq, first_wr, nwr) of the batch last
    mirrored at entry e; returns (batch, steps)."""
    b = hint
    if pub > STREAM_RING and b < pub - STREAM_RING:
        b = pub - STREAM_RING
    for i in range(3 * STREAM_RING):
        seq, first, nwr = ring[b % STREAM_RING]
        if seq == b and w < first + nwr:
            return b, i
        b += 1
    raise AssertionError("walk exceeded three passes of the ring")


def test_piece_rows_rule():
    assert stream_piece_rows(1000, 0, 0, 6) == 1           # first claim: one wave-row
    assert stream_piece_rows(10 ** 6, 3071, 1, 6) == 6      # a backlog: rmax
    assert stream_piece_rows(3071 * 3, 3071 * 10, 10, 6) == 3  # a fair share of the rest
    assert stream_piece_rows(100, 3071 * 10, 30, 6) == 1    # the tail: single wave-rows
    # a wave that did 3x the average work gets 3x the piece
    assert stream_piece_rows(3071 * 2, 3071 * 10, 30, 6) == 6


def test_adaptive_claims_drain_together():
    """Waves progressing at 1 : 0.3 : 0.05 (a SIMD's three waves) over a
    fully published table: with the adaptive rule the last piece of the
    slowest wave ends close to the others' (the tail is a small fraction of
    the run), where equal pieces would leave the slow wave's rmax piece."""
    speeds = [1.0, 0.3, 0.05] * 64
    total, rmax = 20000, 6
    claimed = 0
    mine = [0] * len(speeds)
    free_at = [0.0] * len(speeds)
    while claimed < total:
        w = min(range(len(speeds)), key=lambda i: free_at[i])
        r = min(stream_piece_rows(total - claimed, claimed, mine[w], rmax), total - claimed)
        claimed += r
        mine[w] += r
        free_at[w] += r / speeds[w]
    ideal = total / sum(speeds)
    assert max(free_at) < 1.15 * ideal


def test_ring_lookup_out_of_order_completion():
    rng = random.Random(7)
    ring = [(None, 0, 0)] * STREAM_RING
    first = []          # first wave-row of each batch
    nwr = []
    done = set()
    pub = 0
    wr = 0
    max_steps = 0
    for step in range(20000):
        # publish while the rule allows (X - RING done), up to a random depth
        while rng.random() < 0.6 and (pub < STREAM_RING or (pub - STREAM_RING) in done):
            n = rng.randint(1, 12)
            first.append(wr)
            nwr.append(n)
            ring[pub % STREAM_RING] = (pub, wr, n)
            wr += n
            pub += 1
        live = [b for b in range(max(0, pub - STREAM_RING), pub) if b not in done]
        if not live:
            continue
        # a wave looks up a wave-row of a live batch, from a stale hint and a
        # pub up to one poller pass behind
        b = rng.choice(live)
        w = first[b] + rng.randrange(nwr[b])
        hint = rng.choice([0, max(0, b - rng.randint(0, 3 * STREAM_RING)), b])
        seen_pub = max(b + 1, pub - rng.randint(0, STREAM_RING))
        got, steps = batch_of(ring, seen_pub, hint, w)
        assert got == b
        max_steps = max(max_steps, steps)
        # complete a random live batch (out of order)
        done.add(rng.choice(live))
    assert pub > 10 * STREAM_RING  # the ring wrapped many times
    assert max_steps <= 3 * STREAM_RING


def test_walk_from_hint_alone_misses_after_wraps():
    """The bound the lookup had before the pub lower bound: a first hint of
    0 and two passes of the ring do not reach a batch >= 2 * STREAM_RING."""
    ring = [(None, 0, 0)] * STREAM_RING
    for b in range(150):
        ring[b % STREAM_RING] = (b, b, 1)
    b, w = 0, 140
    for _ in range(2 * STREAM_RING):
        seq, first, n = ring[b % STREAM_RING]
        if seq == b and w < first + n:
            break
        b += 1
    assert b != 140
    assert batch_of(ring, 150, 0, w) == (140, 140 - (150 - STREAM_RING))


def test_idle_exit_and_relaunch_process_every_row_once():
    """The elastic protocol replayed with random interleavings: waves claim
    with a single fetch-and-add while published rows are unclaimed (so
    concurrent claims pass pub_wr), process only the published part of a
    ticket, and drop the rest when the poller declares the kernel idle; every
    launch hands worker w its first ticket at the mirrored pub_wr + w and
    starts the claim counter past those.  Over many
    publish / stall / relaunch cycles every published wave-row is processed
    exactly once and nothing past the published rows ever is."""
    rng = random.Random(11)
    for trial in range(40):
        nwaves = rng.randint(1, 12)
        processed = {}
        pub_wr = 0        # the kernel's mirror (final while idle)
        host_wr = 0       # rows the host has published
        ticket = 0
        launches = 0
        for cycle in range(rng.randint(1, 8)):
            host_wr += rng.randint(1, 60)
            # (re)launch: k_stream_start resets the claim counter past the
            # workers' first tickets, one wave-row each at pub_wr + w
            ticket = pub_wr + nwaves
            launches += 1
            waves = [(pub_wr + w, 1) for w in range(nwaves)]      # (tk, tr) tickets
            mine = [1] * nwaves
            idle = False
            steps = 0
            while True:
                steps += 1
                # the poller mirrors what the host published (sometimes late)
                if not idle and rng.random() < 0.3:
                    pub_wr = host_wr
                active = False
                for w in rng.sample(range(nwaves), nwaves):
                    if waves[w] is None and not idle and pub_wr > ticket:
                        tr = max(1, min(rng.randint(1, 6), pub_wr - ticket))
                        # fetch-and-add: other waves may have read the same `ticket`
                        waves[w] = (ticket, tr + rng.choice([0, 0, 0, 3]))
                        ticket += waves[w][1]
                        mine[w] += waves[w][1]
                    if waves[w] is not None:
                        tk, tr = waves[w]
                        if tk < pub_wr:
                            cnt = min(tr, pub_wr - tk)
                            for r in range(tk, tk + cnt):
                                processed[r] = processed.get(r, 0) + 1
                            waves[w] = (tk + cnt, tr - cnt) if tr > cnt else None
                            active = True
                        elif idle:
                            waves[w] = None  # unpublished rest dropped
                # the poller: idle once everything published is claimed and mirrored
                if not idle and ticket >= pub_wr and pub_wr == host_wr and rng.random() < 0.5:
                    idle = True
                if idle and all(x is None for x in waves):
                    break
                assert steps < 10000
            assert all(r < pub_wr for r in processed)
        # each cycle ends idle only with everything published mirrored and
        # claimed, and the claimed published parts processed
        assert all(processed.get(r) == 1 for r in range(host_wr)), trial
        assert launches >= 1
