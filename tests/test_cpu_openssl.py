"""CPU: the OpenSSL CPU baseline (tools/cpu_openssl: the reference's row
pipeline on OpenSSL 3's secp256k1 arithmetic, bench.py's
`cpu_baseline_openssl`) computes the reference's values and flags.  Its curve
arithmetic is independent of the oracle and of the product, so agreeing with
the stage KATs (numbers held in the reference's own scripts, SURVEY.md
Appendix A), the SQL cases (test/sql/cudasp.test) and the oracle on
synthetic rows pins all three to a third party.  Cases whose spend or label
key is not on the curve (the SQL file's big-endian G, line 66) are outside
what OpenSSL can hold: the baseline refuses them (-2) and they are skipped."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

import golden_io

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "tools", "cpu_openssl", "libcudasp_cpu_openssl.so")


P_FIELD = 2**256 - 2**32 - 977


def on_curve(le64):
    x, y = int.from_bytes(le64[:32], "little"), int.from_bytes(le64[32:], "little")
    return x < P_FIELD and y < P_FIELD and (y * y - x ** 3 - 7) % P_FIELD == 0


def keys_on_curve(spend_hex, label_hexes):
    return all(on_curve(bytes.fromhex(h)) for h in [spend_hex] + list(label_hexes))


@pytest.fixture(scope="module")
def ossl():
    if not os.path.exists(LIB):
        subprocess.check_call(["make", "-s", "-C", os.path.dirname(LIB)])
    lib = ctypes.CDLL(LIB)
    P = ctypes.c_void_p
    lib.cudasp_cpu_openssl_scan.argtypes = [P, P, P, ctypes.c_uint32, P, ctypes.c_uint32, P, P, P, P, ctypes.c_int]
    lib.cudasp_cpu_openssl_scan.restype = ctypes.c_int
    lib.cudasp_cpu_openssl_values.argtypes = [P, P, P, ctypes.c_uint32, P, ctypes.c_uint32, P, P, P, ctypes.c_int]
    lib.cudasp_cpu_openssl_values.restype = ctypes.c_int

    class L:
        @staticmethod
        def scan(scan_key, spend, labels, tweaks, outs, offs, lens, threads=4):
            tw = np.ascontiguousarray(tweaks, dtype=np.uint8)
            outs = np.ascontiguousarray(outs, dtype=np.int64)
            offs = np.ascontiguousarray(offs, dtype=np.uint32)
            lens = np.ascontiguousarray(lens, dtype=np.uint32)
            n = tw.shape[0]
            flags = np.zeros(n, dtype=np.uint8)
            lab = b"".join(labels) if labels else None
            rc = lib.cudasp_cpu_openssl_scan(scan_key, spend, lab, len(labels), tw.ctypes.data, n,
                                             outs.ctypes.data if outs.size else None, offs.ctypes.data,
                                             lens.ctypes.data, flags.ctypes.data, threads)
            return rc, flags

        @staticmethod
        def values(scan_key, spend, labels, tweaks, threads=4):
            tw = np.ascontiguousarray(tweaks, dtype=np.uint8)
            n = tw.shape[0]
            sx = np.zeros((n, 32), dtype=np.uint8)
            t = np.zeros((n, 32), dtype=np.uint8)
            vals = np.zeros((n, 1 + len(labels)), dtype=np.int64)
            lab = b"".join(labels) if labels else None
            rc = lib.cudasp_cpu_openssl_values(scan_key, spend, lab, len(labels), tw.ctypes.data, n, sx.ctypes.data,
                                               t.ctypes.data, vals.ctypes.data, threads)
            return rc, sx, t, vals
    return L


def test_stage_kats(ossl):
    """S.x, the tagged hash and v (base and label) of the KAT rows."""
    kats = golden_io.load("stage_kats.json")
    checked = 0
    for k in kats:
        labels = [bytes.fromhex(l) for l in k["label_keys"]]
        tw = golden_io.tweak_array([k["tweak"]])
        rc, sx, t, vals = ossl.values(bytes.fromhex(k["scan_key"]), bytes.fromhex(k["spend_key"]), labels, tw, 1)
        if not keys_on_curve(k["spend_key"], k["label_keys"]):
            assert rc == -2  # OpenSSL refuses the key; the reference runs its formulas on it
            continue
        assert rc == 0
        checked += 1
        assert sx[0].tobytes().hex() == k["S_x"], k["height"]
        assert t[0].tobytes().hex() == k["t"], k["height"]
        assert int(vals[0, 0]) == k["v"], k["height"]
        assert [int(v) for v in vals[0, 1:]] == k["label_values"], k["height"]
    assert checked == len(kats) - 1  # height 100 under the big-endian G of line 66


def test_sql_cases(ossl):
    """Every query of test/sql/cudasp.test: the rows the OpenSSL pipeline
    flags give the query's expected result."""
    sc = golden_io.load("sql_cases.json")
    checked = 0
    for q in sc["queries"]:
        if q["table"] == "test_data":
            visible = sc["tables"]["test_data"][:q["test_data_rows_visible"]]
            rows = [r for r in visible if q["where_height"] in (None, r["height"])]
            mult = 1
        else:
            rows = [sc["tables"][q["table"]]["row"]]
            mult = sc["tables"][q["table"]]["repeat"]
        tw = golden_io.tweak_array([r["tweak"] for r in rows])
        outs, offs, lens = golden_io.csr([r["outputs"] for r in rows])
        labels = [bytes.fromhex(l) for l in q["label_keys"]]
        rc, flags = ossl.scan(bytes.fromhex(q["scan_key"]), bytes.fromhex(q["spend_key"]), labels, tw, outs, offs,
                              lens)
        if not keys_on_curve(q["spend_key"], q["label_keys"]):
            assert rc == -2, q["line"]
            continue
        assert rc == 0, q["line"]
        checked += 1
        hit = [r for r, f in zip(rows, flags) if f] * mult
        got = [len(hit)] if q["select"] == "count" else sorted(r["height"] for r in hit)
        assert got == q["expected"], q["line"]
    assert checked == len(sc["queries"]) - 1  # line 66


def test_random_rows_fixture(ossl):
    rr = golden_io.load("random_rows.json")
    rows = rr["rows"]
    scan, spend = bytes.fromhex(rr["scan_key"]), bytes.fromhex(rr["spend_key"])
    labels = [bytes.fromhex(l) for l in rr["label_keys"]]
    tw = golden_io.tweak_array([r["tweak"] for r in rows])
    outs, offs, lens = golden_io.csr([r["outputs"] for r in rows])
    for L, key in ((len(labels), "match_all_labels"), (0, "match_no_labels"), (1, "match_first_label")):
        rc, got = ossl.scan(scan, spend, labels[:L], tw, outs, offs, lens)
        assert rc == 0
        assert got.tolist() == [int(r[key]) for r in rows], key


def test_synthetic_values_vs_oracle(ossl):
    """bench's synthetic tweaks and 16 label keys: every value equals the C
    oracle's (row counts not a multiple of the worker blocks)."""
    import sys
    sys.path.insert(0, ROOT)
    import bench
    from oracle import oracle
    labels = bench.label_keys(16)
    s0 = bench.synth_s0()
    n = 131
    tw = np.frombuffer(b"".join(oracle.synth_tweak(s0, 7000 + i) for i in range(n)), dtype=np.uint8).reshape(n, 64)
    _, want = oracle.scan(bench.SCAN_KEY, bench.SPEND_KEY, labels, tw, threads=4, want_values=True)
    rc, _, _, got = ossl.values(bench.SCAN_KEY, bench.SPEND_KEY, labels, tw, threads=3)
    assert rc == 0
    assert (got == want).all()


def test_off_curve_rows_refused(ossl):
    """A tweak off the curve is refused (flag 0, counted), not guessed."""
    rr = golden_io.load("random_rows.json")
    tw = golden_io.tweak_array([r["tweak"] for r in rr["rows"][:3]]).copy()
    tw[1, 40] ^= 1
    outs, offs, lens = golden_io.csr([r["outputs"] for r in rr["rows"][:3]])
    rc, flags = ossl.scan(bytes.fromhex(rr["scan_key"]), bytes.fromhex(rr["spend_key"]), [], tw, outs, offs, lens)
    assert rc == 1
    assert flags[1] == 0
