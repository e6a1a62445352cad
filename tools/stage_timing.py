"""Isolated per-stage timing (HIP events, one stream) at a batch of n rows,
on random tweak words, for A/B comparison of library builds (CUDASP_LIB)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "duckdb-cudasp-extension_amd"))
from cudasp_amd import Scanner  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 300000
L = int(sys.argv[2]) if len(sys.argv) > 2 else 0
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
scan = bytes.fromhex("2c1f0cb94db3946522cc1487256535dd33a1f911946baff817a72880064e690f")
spend = bytes.fromhex("36cf8fcd4d4890ab6c1083aeb5b50c260c20acda7839120e3575836f6d85c95ce0d705e31ff9fdcce67a8f3598871c6dfbe6bcde8a51cb7b48b0f95be0ea94de")
s = Scanner(scan, spend, [spend] * L, max_rows=n)
g = torch.Generator(device="cuda").manual_seed(1)
tx = torch.randint(-2**31, 2**31 - 1, (8, n), dtype=torch.int32, device="cuda", generator=g)
ty = torch.randint(-2**31, 2**31 - 1, (8, n), dtype=torch.int32, device="cuda", generator=g)
outs = torch.randint(-2**62, 2**62, (2 * n,), dtype=torch.int64, device="cuda", generator=g)
offs = torch.arange(n, dtype=torch.int32, device="cuda") * 2
lens = torch.full((n,), 2, dtype=torch.int32, device="cuda")
flags = torch.zeros(n, dtype=torch.uint8, device="cuda")
t = torch.empty((8 * n,), dtype=torch.int32, device="cuda")
st = torch.cuda.Stream()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(3 * reps)]
for _ in range(2):
    s.stage_shared_secret(tx, ty, n, st, t_out=t)
    s.stage_match(outs, offs, lens, n, flags, stream=st, t_in=t)
for i in range(reps):
    ev[3 * i].record(st)
    s.stage_shared_secret(tx, ty, n, st, t_out=t)
    ev[3 * i + 1].record(st)
    s.stage_match(outs, offs, lens, n, flags, stream=st, t_in=t)
    ev[3 * i + 2].record(st)
torch.cuda.synchronize()
a = sorted(ev[3 * i].elapsed_time(ev[3 * i + 1]) for i in range(reps))
b = sorted(ev[3 * i + 1].elapsed_time(ev[3 * i + 2]) for i in range(reps))
lib = os.path.basename(os.environ.get("CUDASP_LIB", "libcudasp_amd.so"))
print("%-22s n=%d L=%d  stageA %.3f ms (min %.3f)  stageB %.3f ms (min %.3f)  -> %.2f M rows/s" % (
    lib, n, L, a[reps // 2], a[0], b[reps // 2], b[0], n / (a[reps // 2] + b[reps // 2]) / 1e3), flush=True)
s.close()
