"""Count gfx950 instructions per probe kernel (tools/isa/fe_ops.hip).

    python tools/isa/isa_count.py [-DCUDASP_FE_VARIANT=0 ...]

Prints, per kernel, the total instruction count, VALU count and the VALU
mnemonic histogram minus the load/store probe's, so each line is the cost of
the operation itself.  Static counts (straight-line code); loops in an
operation (safegcd) are reported as their static size.
"""
import collections
import os
import re
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))


def compile_asm(extra):
    out = os.path.join(tempfile.gettempdir(), "fe_ops_%d.s" % os.getpid())
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-S",
           "-o", out, os.path.join(HERE, "fe_ops.hip")] + extra
    subprocess.check_call(cmd)
    text = open(out).read()
    os.unlink(out)
    return text


def parse(text):
    kernels = {}
    cur = None
    for line in text.splitlines():
        m = re.match(r"^(probe_\w+):", line)
        if m:
            cur = kernels.setdefault(m.group(1), collections.Counter())
            continue
        if cur is None:
            continue
        if line.startswith("\ts_endpgm"):
            cur["s_endpgm"] += 1
            cur = None
            continue
        s = line.strip()
        if not s or s.startswith((";", ".", "//")) or s.endswith(":"):
            continue
        cur[s.split()[0]] += 1
    return kernels


def main():
    ks = parse(compile_asm(sys.argv[1:]))
    base = ks.get("probe_loadstore", collections.Counter())
    for name, c in ks.items():
        if name == "probe_loadstore":
            continue
        valu = {k: v for k, v in c.items() if k.startswith("v_")}
        nvalu = sum(valu.values()) - sum(v for k, v in base.items() if k.startswith("v_"))
        tot = sum(c.values()) - sum(base.values())
        top = sorted(((v - base.get(k, 0), k) for k, v in valu.items()), reverse=True)[:10]
        nops = c.get("s_nop", 0)
        print("%-12s total %5d  valu %5d  s_nop %3d  | %s" % (name, tot, nvalu, nops,
              " ".join("%s:%d" % (k, v) for v, k in top)))


if __name__ == "__main__":
    main()
