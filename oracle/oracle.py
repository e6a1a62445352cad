"""ctypes face of the C oracle (oracle/cudasp_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, as the checker -- never by the product path.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "libcudasp_oracle.so")
LABEL_INFINITY = -(1 << 63)

_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        lib = ctypes.CDLL(LIB)
        P = ctypes.c_void_p
        lib.cudasp_oracle_row.argtypes = [P, P, P, ctypes.c_uint32, P, P, P]
        lib.cudasp_oracle_row.restype = ctypes.c_int
        lib.cudasp_oracle_scan.argtypes = [P, P, P, ctypes.c_uint32, P, ctypes.c_uint32, P, P, P, P, P, ctypes.c_int]
        lib.cudasp_oracle_scan.restype = ctypes.c_int
        lib.cudasp_oracle_row_ex.argtypes = [P, P, P, ctypes.c_uint32, P, P, P, P, P]
        lib.cudasp_oracle_row_ex.restype = ctypes.c_int
        lib.cudasp_oracle_scan_ex.argtypes = [P, P, P, ctypes.c_uint32, P, ctypes.c_uint32, P, P, P, P, P, P,
                                              ctypes.c_int]
        lib.cudasp_oracle_scan_ex.restype = ctypes.c_int
        lib.cudasp_oracle_synth_tweak.argtypes = [P, ctypes.c_uint64, P]
        lib.cudasp_oracle_synth_tweak.restype = ctypes.c_int
        lib.cudasp_oracle_sha256.argtypes = [P, P, ctypes.c_size_t]
        lib.cudasp_oracle_fp_mul.argtypes = [P, P, P]
        _lib = lib
    return _lib


def row(scan, spend, labels, tweak):
    """-> (t as 32 BE bytes, [v_base, v_label_0, ...])"""
    lib = load()
    L = len(labels)
    t = ctypes.create_string_buffer(32)
    vals = (ctypes.c_int64 * (1 + L))()
    lab = b"".join(labels) if labels else None
    rc = lib.cudasp_oracle_row(scan, spend, lab, L, tweak, t, vals)
    if rc != 0:
        raise ValueError("degenerate row (point at infinity)")
    return t.raw, list(vals)


def scan(scan_key, spend_key, labels, tweaks, outputs=None, offsets=None, lengths=None, threads=1,
         want_values=False):
    """Vectorised oracle over n rows.  tweaks: uint8 [n, 64].  Returns
    (flags uint8 [n] or None, values int64 [n, 1+L] or None)."""
    lib = load()
    tw = np.ascontiguousarray(tweaks, dtype=np.uint8).reshape(-1, 64)
    n = tw.shape[0]
    L = len(labels)
    lab = b"".join(labels) if labels else None
    flags = None
    if outputs is not None:
        outputs = np.ascontiguousarray(outputs, dtype=np.int64)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint32)
        lengths = np.ascontiguousarray(lengths, dtype=np.uint32)
        flags = np.zeros(n, dtype=np.uint8)
    values = np.zeros((n, 1 + L), dtype=np.int64) if want_values else None
    ptr = lambda a: None if a is None else a.ctypes.data
    outs_ptr = ptr(outputs) if (outputs is not None and outputs.size) else None
    lib.cudasp_oracle_scan(scan_key, spend_key, lab, L, ptr(tw), n, outs_ptr, ptr(offsets), ptr(lengths),
                           ptr(flags), ptr(values), int(threads))
    return flags, values


class _Options(ctypes.Structure):
    _fields_ = [("output_count", ctypes.c_uint32), ("label_negation", ctypes.c_uint32),
                ("full_x", ctypes.c_uint32)]


def row_ex(scan, spend, labels, tweak, output_count=1, label_negation=False):
    """-> (K digests (32 BE bytes each), values [K][1 + L'], xs [K][1 + L'] as
    32-byte BE x or None at infinity) for the protocol variants."""
    lib = load()
    L = len(labels)
    W = 1 + (2 if label_negation else 1) * L
    K = output_count
    opt = _Options(K, int(bool(label_negation)), 0)
    t = ctypes.create_string_buffer(32 * K)
    xs = ctypes.create_string_buffer(32 * K * W)
    vals = (ctypes.c_int64 * (K * W))()
    lab = b"".join(labels) if labels else None
    if lib.cudasp_oracle_row_ex(scan, spend, lab, L, tweak, ctypes.byref(opt), t, xs, vals) != 0:
        raise ValueError("degenerate row (point at infinity)")
    v = [list(vals[k * W:(k + 1) * W]) for k in range(K)]
    x = [[None if v[k][c] == LABEL_INFINITY and c else xs.raw[32 * (k * W + c):32 * (k * W + c + 1)]
          for c in range(W)] for k in range(K)]
    return [t.raw[32 * k:32 * (k + 1)] for k in range(K)], v, x


def scan_ex(scan_key, spend_key, labels, tweaks, outputs=None, offsets=None, lengths=None, output_count=1,
            label_negation=False, full_x=False, threads=1, want_values=False):
    """scan() for the protocol variants: outputs are int64 values, or with
    full_x a uint8 [total, 32] array of BE x-only keys.  values: int64
    [n, K, 1 + L']."""
    lib = load()
    tw = np.ascontiguousarray(tweaks, dtype=np.uint8).reshape(-1, 64)
    n = tw.shape[0]
    L = len(labels)
    W = 1 + (2 if label_negation else 1) * L
    lab = b"".join(labels) if labels else None
    opt = _Options(output_count, int(bool(label_negation)), int(bool(full_x)))
    flags = None
    if outputs is not None:
        outputs = np.ascontiguousarray(outputs, dtype=np.uint8 if full_x else np.int64)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint32)
        lengths = np.ascontiguousarray(lengths, dtype=np.uint32)
        flags = np.zeros(n, dtype=np.uint8)
    values = np.zeros((n, output_count, W), dtype=np.int64) if want_values else None
    ptr = lambda a: None if a is None else a.ctypes.data
    outs_ptr = ptr(outputs) if (outputs is not None and outputs.size) else None
    lib.cudasp_oracle_scan_ex(scan_key, spend_key, lab, L, ptr(tw), n, ctypes.byref(opt), outs_ptr, ptr(offsets),
                              ptr(lengths), ptr(flags), ptr(values), int(threads))
    return flags, values


def synth_tweak(s0_le, index):
    out = ctypes.create_string_buffer(64)
    if load().cudasp_oracle_synth_tweak(s0_le, index, out) != 0:
        raise ValueError("synthetic tweak at infinity")
    return out.raw


def sha256(msg):
    out = ctypes.create_string_buffer(32)
    load().cudasp_oracle_sha256(out, msg, len(msg))
    return out.raw


def fp_mul(a, b):
    out = ctypes.create_string_buffer(32)
    load().cudasp_oracle_fp_mul(a, b, out)
    return out.raw


def check_planted_sample(sample, threads=1):
    """Checker of an end-to-end run's row sample (tools/host_e2e
    --plant-sample: planted and unplanted rows strided over the table, with
    the keys and what the run emitted).  Every row is recomputed here:
    its tweak must be the synthetic generator's T_g = (s0 + g) G, a planted
    row's planted value (its first output) must be the oracle's value of
    its column (0 = base, 1 + j = label j) and its oracle flag 1, an
    unplanted row's oracle flag 0, and the run must have emitted exactly
    the rows the oracle flags.  Returns {rows, equal, planted, unplanted,
    mismatches (first few)}; equal == rows means the sample agrees."""
    scan_key = bytes.fromhex(sample["scan"])
    spend_key = bytes.fromhex(sample["spend"])
    labels = [bytes.fromhex(h) for h in sample["labels"]]
    s0 = bytes.fromhex(sample["s0_le"])
    rows = sample["rows"]
    n = len(rows)
    if n == 0:
        return dict(rows=0, equal=0, planted=0, unplanted=0, mismatches=[])
    tw = np.frombuffer(b"".join(bytes.fromhex(r["tweak"]) for r in rows), dtype=np.uint8).reshape(n, 64)
    lens = np.array([len(r["outputs"]) for r in rows], dtype=np.uint32)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint32)
    outs = np.array([v for r in rows for v in r["outputs"]], dtype=np.int64)
    flags, vals = scan(scan_key, spend_key, labels, tw, outs, offs, lens, threads=threads, want_values=True)
    equal, bad = 0, []
    for i, r in enumerate(rows):
        ok = bytes(tw[i]) == synth_tweak(s0, r["g"])
        if r["column"] >= 0:
            ok = ok and len(r["outputs"]) > 0 and int(vals[i, r["column"]]) == r["outputs"][0] and flags[i] == 1
        else:
            ok = ok and flags[i] == 0
        ok = ok and int(flags[i]) == int(r["emitted"])
        equal += ok
        if not ok and len(bad) < 8:
            bad.append(dict(g=r["g"], column=r["column"], emitted=r["emitted"], oracle_flag=int(flags[i])))
    planted = sum(1 for r in rows if r["column"] >= 0)
    return dict(rows=n, equal=equal, planted=planted, unplanted=n - planted,
                label_columns=sorted({r["column"] for r in rows if r["column"] > 0}), mismatches=bad)
