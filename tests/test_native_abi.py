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
