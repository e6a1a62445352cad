"""GPU: the library and torch share one HIP runtime whichever initialises the
GPU first (the Makefile's HIPRT_LINK; round-5 verdict item 5).

tools/probes/init_order.py makes the library's HIP calls first -- a
NativePinnedTable created and appended before torch is even imported, as a
DuckDB host or a C++ caller would -- and then asks torch for the device and a
tensor on it.  With the library linked against the runtime's soname, torch
loaded a second runtime there and found no GPU."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_first_then_torch():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "probes", "init_order.py")],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    out = r.stdout
    assert "native created" in out and "torch tensor ok cuda:0" in out, out
    assert "available True" in out, out
