"""CPU: the C-ABI library loads and exports every symbol the headers in
include/ declare; without a device every entry point fails loudly."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INCLUDE = os.path.join(ROOT, "include")


def declared_functions():
    names = set()
    for h in os.listdir(INCLUDE):
        if not h.endswith(".h"):
            continue
        text = open(os.path.join(INCLUDE, h)).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        for m in re.finditer(r"^[A-Za-z_][\w\s\*]*?\b(\w+)\s*\(", text, flags=re.M):
            name = m.group(1)
            if name not in ("defined",):
                names.add(name)
    return sorted(names)


def test_headers_declare_the_reference_abi():
    names = declared_functions()
    for n in ("LaunchBatchScan", "RunBatchScanKernels", "FreeBatchScanState", "cudasp_scanner_create",
              "cudasp_scan_device", "cudasp_tf_bind", "cudasp_tf_final"):
        assert n in names


def test_library_exports_every_declared_symbol():
    from cudasp_amd import _native
    lib = _native.load()
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert missing == []


def test_no_device_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("device present")
    from cudasp_amd import CudaspError, Scanner
    from cudasp_amd import _native
    assert _native.load().cudasp_device_count() == 0
    with pytest.raises(CudaspError) as e:
        Scanner(b"\x01" * 32, b"\x02" * 64, [], max_rows=16)
    assert e.value.code == _native.CUDASP_ERR_NO_DEVICE


def test_version_string():
    from cudasp_amd import _native
    assert b"gfx950" in _native.load().cudasp_version()


def test_prepared_device_batches_match_the_abi_struct():
    """Scanner.device_batches builds the cudasp_device_batch array once (the
    bench's step reuses it): field order and values as scan_device_batches
    would pass them, references to the tensors held."""
    import torch
    from cudasp_amd import Scanner, _native
    n = 100
    t = {k: torch.zeros(s, dtype=d) for k, s, d in (("tweak_x", 8 * n, torch.int32), ("tweak_y", 8 * n, torch.int32),
                                                   ("outputs", 2 * n, torch.int64), ("offsets", n, torch.int32),
                                                   ("lengths", n, torch.int32), ("flags", n, torch.uint8),
                                                   ("match_rows", n, torch.int32), ("match_count", 1, torch.int32))}
    prep = Scanner.device_batches([t, dict(t, flags=t["flags"][:7])])
    assert prep.count == 2 and isinstance(prep.array[0], _native.DeviceBatch)
    names = [f[0] for f in _native.DeviceBatch._fields_]
    b0 = prep.array[0]
    want = dict(zip(names, (t["tweak_x"].data_ptr(), t["tweak_y"].data_ptr(), t["outputs"].data_ptr(),
                            t["offsets"].data_ptr(), t["lengths"].data_ptr(), n, t["flags"].data_ptr(),
                            t["match_rows"].data_ptr(), t["match_count"].data_ptr())))
    assert {k: getattr(b0, k) for k in names} == want
    assert getattr(prep.array[1], names[5]) == 7
    assert len(Scanner.device_batches([]).array) == 1 and Scanner.device_batches([]).count == 0


def _dt_needed(path):
    """DT_NEEDED names of an ELF64 shared object."""
    import struct
    d = open(path, "rb").read()
    shoff, = struct.unpack_from("<Q", d, 0x28)
    shentsize, shnum, _ = struct.unpack_from("<HHH", d, 0x3A)
    secs = [struct.unpack_from("<IIQQQQIIQQ", d, shoff + i * shentsize) for i in range(shnum)]
    out = []
    for name, typ, flags, addr, off, size, link, info, align, entsize in secs:
        if typ != 6:  # SHT_DYNAMIC
            continue
        stroff = secs[link][4]
        for i in range(size // 16):
            tag, val = struct.unpack_from("<qQ", d, off + 16 * i)
            if tag == 1:  # DT_NEEDED
                out.append(d[stroff + val:d.index(b"\0", stroff + val)].decode())
    return out


def test_library_names_the_hip_runtime_like_torch():
    """The library depends on the HIP runtime by its unversioned file name,
    the name torch's libraries use, so both bind one runtime in either load
    order (Makefile, HIPRT_LINK)."""
    from cudasp_amd import _native
    needed = _dt_needed(_native.LIB_PATH)
    assert "libamdhip64.so" in needed, needed
    assert "libamdhip64.so.7" not in needed, needed


_MAPS_PROBE = r"""
import ctypes, os, sys
sys.path.insert(0, %r)
order = sys.argv[1]
if order == "torch-first":
    import torch
from cudasp_amd import _native
_native.load()
if order == "lib-first":
    import torch
    torch.cuda.device_count()
maps = {l.split()[-1] for l in open("/proc/self/maps") if "libamdhip64" in l}
print(sorted({os.path.realpath(m) for m in maps}))
"""


@pytest.mark.parametrize("order", ["lib-first", "torch-first"])
def test_one_hip_runtime_in_either_load_order(order):
    """A process that loads the library before torch (a DuckDB host, a
    NativePinnedTable) and one that imports torch first both map exactly one
    HIP runtime file."""
    import ast
    import subprocess
    import sys
    pkg = os.path.join(ROOT, "duckdb-cudasp-extension_amd")
    r = subprocess.run([sys.executable, "-c", _MAPS_PROBE % pkg, order], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    files = ast.literal_eval(r.stdout.strip().splitlines()[-1])
    assert len(files) == 1, files
