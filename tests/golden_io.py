"""Helpers to turn the committed golden fixtures into arrays."""
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def csr(outputs_lists):
    """Flatten per-row outputs lists with the reference's NULL rules
    (src/cudasp_extension.cu:206-221): a NULL list gives length 0, NULL
    elements are dropped."""
    vals, offs, lens = [], [], []
    for o in outputs_lists:
        offs.append(len(vals))
        kept = [x for x in (o or []) if x is not None]
        vals.extend(kept)
        lens.append(len(kept))
    return (np.array(vals, dtype=np.int64), np.array(offs, dtype=np.uint32), np.array(lens, dtype=np.uint32))


def tweak_array(hex_list):
    return np.frombuffer(b"".join(bytes.fromhex(h) for h in hex_list), dtype=np.uint8).reshape(-1, 64)


def tweak_columns(tweaks):
    """[n, 64] LE blobs -> (x, y) column-major u32 arrays of shape [8, n]."""
    w = np.ascontiguousarray(tweaks).view("<u4").reshape(-1, 16)
    return np.ascontiguousarray(w[:, :8].T), np.ascontiguousarray(w[:, 8:].T)
