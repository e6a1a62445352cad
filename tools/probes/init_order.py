"""Probe: does torch's CUDA init still work after the library initialised HIP
first (a NativePinnedTable created before any torch.cuda call)?"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "duckdb-cudasp-extension_amd"))
import pyarrow as pa

from cudasp_amd import NativePinnedTable, _native

print("lib device count", _native.load().cudasp_device_count(), flush=True)
t = pa.table({"txid": pa.array([b"t"]), "height": pa.array([1], pa.int32()), "tweak_key": pa.array([bytes(64)]),
              "outputs": pa.array([[1]], pa.list_(pa.int64()))})
with NativePinnedTable(t) as pt:
    print("native created", pt.info()["batches"], flush=True)
import torch

print("torch device_count", torch.cuda.device_count(), "available", torch.cuda.is_available(), flush=True)
x = torch.empty(4, device="cuda:0")
print("torch tensor ok", x.device, flush=True)
