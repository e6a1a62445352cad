"""Print VGPR/SGPR/scratch/occupancy per kernel of scan_kernels.hip (hipcc remarks)."""
import re
import subprocess
import sys

src = sys.argv[1] if len(sys.argv) > 1 else "duckdb-cudasp-extension_amd/csrc/scan_kernels.hip"
extra = sys.argv[2:]
out = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-c", "-o", "/tmp/ru.o", src,
                      "-Rpass-analysis=kernel-resource-usage"] + extra, capture_output=True, text=True).stderr
cur = None
rows = {}
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+([A-Za-z \[\]/]+?): (\d+)", line)
    if m and cur:
        rows[cur][m.group(1).strip()] = int(m.group(2))
for k, v in rows.items():
    print("%-60s VGPR %3s AGPR %3s SGPR %3s scratch %4s occ %s spillV %s" % (
        k[:60], v.get("VGPRs"), v.get("AGPRs"), v.get("SGPRs"), v.get("ScratchSize [bytes/lane]"),
        v.get("Occupancy [waves/SIMD]"), v.get("VGPRs Spill")))
