"""CPU: the optimized CPU baseline (tools/cpu_port: the product's row pipeline
compiled for the host at -O3, bench.py's `cpu_baseline_optimized`) computes
the reference's flags -- equal to the C oracle's and to the golden fixtures
-- so the baseline it times is the same work."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

import golden_io

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "tools", "cpu_port", "libcudasp_cpu_port.so")


@pytest.fixture(scope="module")
def port():
    if not os.path.exists(LIB):
        subprocess.check_call(["make", "-s", "-C", os.path.dirname(LIB)])
    lib = ctypes.CDLL(LIB)
    P = ctypes.c_void_p
    lib.cudasp_cpu_port_scan.argtypes = [P, P, P, ctypes.c_uint32, P, ctypes.c_uint32, P, P, P, P, ctypes.c_int]
    lib.cudasp_cpu_port_scan.restype = ctypes.c_int

    def scan(scan_key, spend, labels, tweaks, outs, offs, lens, threads=4):
        tw = np.ascontiguousarray(tweaks, dtype=np.uint8)
        outs = np.ascontiguousarray(outs, dtype=np.int64)
        offs = np.ascontiguousarray(offs, dtype=np.uint32)
        lens = np.ascontiguousarray(lens, dtype=np.uint32)
        n = tw.shape[0]
        flags = np.zeros(n, dtype=np.uint8)
        lab = b"".join(labels) if labels else None
        rc = lib.cudasp_cpu_port_scan(scan_key, spend, lab, len(labels), tw.ctypes.data, n,
                                      outs.ctypes.data if outs.size else None, offs.ctypes.data, lens.ctypes.data,
                                      flags.ctypes.data, threads)
        assert rc == 0
        return flags
    return scan


def test_random_rows_fixture(port):
    rr = golden_io.load("random_rows.json")
    rows = rr["rows"]
    scan, spend = bytes.fromhex(rr["scan_key"]), bytes.fromhex(rr["spend_key"])
    labels = [bytes.fromhex(l) for l in rr["label_keys"]]
    tw = golden_io.tweak_array([r["tweak"] for r in rows])
    outs, offs, lens = golden_io.csr([r["outputs"] for r in rows])
    for L, key in ((len(labels), "match_all_labels"), (0, "match_no_labels"), (1, "match_first_label")):
        got = port(scan, spend, labels[:L], tw, outs, offs, lens)
        assert got.tolist() == [int(r[key]) for r in rows], key


def test_synthetic_16_labels_vs_oracle(port):
    import sys
    sys.path.insert(0, ROOT)
    import bench
    from oracle import oracle
    labels = bench.label_keys(16)
    s0 = bench.synth_s0()
    n = 203  # not a multiple of the 8-row groups
    tw = np.frombuffer(b"".join(oracle.synth_tweak(s0, 5000 + i) for i in range(n)), dtype=np.uint8).reshape(n, 64)
    _, vals = oracle.scan(bench.SCAN_KEY, bench.SPEND_KEY, labels, tw, threads=4, want_values=True)
    outs = np.arange(3 * n, dtype=np.int64).reshape(n, 3) * 977
    for i in range(0, n, 3):
        outs[i, 2] = vals[i, (i // 3) % 17]
    offs = np.arange(n, dtype=np.uint32) * 3
    lens = np.full(n, 3, dtype=np.uint32)
    want, _ = oracle.scan(bench.SCAN_KEY, bench.SPEND_KEY, labels, tw, outs.reshape(-1), offs, lens, threads=4)
    assert int(want.sum()) >= n // 3
    got = port(bench.SCAN_KEY, bench.SPEND_KEY, labels, tw, outs.reshape(-1), offs, lens)
    assert (got == want).all()
