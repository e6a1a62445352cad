"""CPU: the C oracle's protocol variants (output indices k > 0, label
negation, full-x compare) against the pure-Python
statement in tests/variants.py.  With the default options the variant entry
points reduce to the pinned reference semantics."""
import numpy as np

import golden_io
import variants as V
from oracle import oracle


def _case(nrows=4):
    rr = golden_io.load("random_rows.json")
    rows = rr["rows"][:nrows]
    return (bytes.fromhex(rr["scan_key"]), bytes.fromhex(rr["spend_key"]),
            [bytes.fromhex(l) for l in rr["label_keys"]], rows)


def test_defaults_are_the_reference():
    scan, spend, labels, rows = _case(8)
    tw = golden_io.tweak_array([r["tweak"] for r in rows])
    outs, offs, lens = golden_io.csr([r["outputs"] for r in rows])
    f0, v0 = oracle.scan(scan, spend, labels, tw, outs, offs, lens, want_values=True)
    f1, v1 = oracle.scan_ex(scan, spend, labels, tw, outs, offs, lens, want_values=True)
    assert (f0 == f1).all() and (v0 == v1[:, 0, :]).all()
    for i, r in enumerate(rows):
        assert int(v1[i, 0, 0]) == r["v"]


def test_row_ex_matches_python_statement():
    scan, spend, labels, rows = _case(3)
    for r in rows:
        tweak = bytes.fromhex(r["tweak"])
        for K, negf in ((1, False), (3, False), (2, True)):
            t, v, x = oracle.row_ex(scan, spend, labels[:2], tweak, output_count=K, label_negation=negf)
            cands, digests = V.row(scan, spend, labels[:2], tweak, K, negf)
            assert t == digests
            assert v == V.values(cands)
            assert x == [[None if p is None else V.x_bytes(p) for p in ks] for ks in cands]


def _planted_table(scan, spend, labels, tweaks, kind):
    """Outputs per row such that row i matches only through variant `kind`
    (and with the default options for kind 'base')."""
    outs_int, outs_x = [], []
    for i, tw in enumerate(tweaks):
        cands, _ = V.row(scan, spend, labels, tw, 3, True)
        L = len(labels)
        pick = {"base": cands[0][0], "k2": cands[2][0], "k1_label": cands[1][1], "neg": cands[0][1 + L],
                "none": V.mul(7 + i, V.G)}[kind]
        outs_int.append([12345, V.upper64(pick[0])])
        outs_x.append([b"\x11" * 32, V.x_bytes(pick)])
    return outs_int, outs_x


def test_variant_flags():
    scan, spend, labels, rows = _case(6)
    labels = labels[:2]
    tweaks = [bytes.fromhex(r["tweak"]) for r in rows]
    tw = golden_io.tweak_array([r["tweak"] for r in rows])
    # expected flag per (kind, options): output_count, label_negation
    expect = {
        "base": {(1, False): 1, (3, False): 1, (1, True): 1, (3, True): 1},
        "k2": {(1, False): 0, (3, False): 1, (1, True): 0, (3, True): 1},
        "k1_label": {(1, False): 0, (3, False): 1, (1, True): 0, (3, True): 1},
        "neg": {(1, False): 0, (3, False): 0, (1, True): 1, (3, True): 1},
        "none": {(1, False): 0, (3, False): 0, (1, True): 0, (3, True): 0},
    }
    for kind, table in expect.items():
        outs_int, outs_x = _planted_table(scan, spend, labels, tweaks, kind)
        oi, offs, lens = golden_io.csr(outs_int)
        ox = np.frombuffer(b"".join(b"".join(o) for o in outs_x), dtype=np.uint8).reshape(-1, 32)
        for (K, negf), want in table.items():
            fi, _ = oracle.scan_ex(scan, spend, labels, tw, oi, offs, lens, output_count=K, label_negation=negf)
            fx, _ = oracle.scan_ex(scan, spend, labels, tw, ox, offs, lens, output_count=K, label_negation=negf,
                                   full_x=True)
            assert list(fi) == [want] * len(rows), (kind, K, negf)
            assert list(fx) == [want] * len(rows), (kind, K, negf)


def test_full_x_rejects_upper64_collisions():
    """An output with the right upper 64 bits but a different x matches in the
    int64 mode (the reference's) and not with full_x."""
    scan, spend, labels, rows = _case(2)
    tweaks = [bytes.fromhex(r["tweak"]) for r in rows]
    tw = golden_io.tweak_array([r["tweak"] for r in rows])
    xs, ints = [], []
    for t in tweaks:
        F = V.row(scan, spend, [], t)[0][0][0]
        x = bytearray(V.x_bytes(F))
        x[31] ^= 1
        xs.append([bytes(x)])
        ints.append([V.upper64(F[0])])
    oi, offs, lens = golden_io.csr(ints)
    ox = np.frombuffer(b"".join(b"".join(o) for o in xs), dtype=np.uint8).reshape(-1, 32)
    fi, _ = oracle.scan_ex(scan, spend, [], tw, oi, offs, lens)
    fx, _ = oracle.scan_ex(scan, spend, [], tw, ox, offs, lens, full_x=True)
    assert list(fi) == [1, 1] and list(fx) == [0, 0]
