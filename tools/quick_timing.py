"""Quick device-resident timing of the scan pipeline on random tweak words
(development probe; bench.py is the measured benchmark)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "duckdb-cudasp-extension_amd"))
from cudasp_amd import Scanner  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 300000
L = int(sys.argv[2]) if len(sys.argv) > 2 else 0
scan = bytes.fromhex("2c1f0cb94db3946522cc1487256535dd33a1f911946baff817a72880064e690f")
spend = bytes.fromhex("36cf8fcd4d4890ab6c1083aeb5b50c260c20acda7839120e3575836f6d85c95ce0d705e31ff9fdcce67a8f3598871c6dfbe6bcde8a51cb7b48b0f95be0ea94de")
labels = [spend] * L
t0 = time.time()
s = Scanner(scan, spend, labels, max_rows=n)
print("scanner create (incl. table build) %.3f s" % (time.time() - t0), flush=True)
g = torch.Generator(device="cuda").manual_seed(1)
tx = torch.randint(-2**31, 2**31 - 1, (8, n), dtype=torch.int32, device="cuda", generator=g)
ty = torch.randint(-2**31, 2**31 - 1, (8, n), dtype=torch.int32, device="cuda", generator=g)
outs = torch.randint(-2**62, 2**62, (2 * n,), dtype=torch.int64, device="cuda", generator=g)
offs = (torch.arange(n, dtype=torch.int32, device="cuda") * 2)
lens = torch.full((n,), 2, dtype=torch.int32, device="cuda")
flags = torch.zeros(n, dtype=torch.uint8, device="cuda")
st = torch.cuda.Stream()
torch.cuda.set_stream(st)
for i in range(2):
    s.scan_device(tx, ty, outs, offs, lens, flags, stream=st)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
reps = 5
e0.record(st)
for i in range(reps):
    s.scan_device(tx, ty, outs, offs, lens, flags, stream=st)
e1.record(st)
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / reps
print("n=%d L=%d: %.3f ms per batch -> %.3f M rows/s" % (n, L, ms, n / ms / 1e3))
