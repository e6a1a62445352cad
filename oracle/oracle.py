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
