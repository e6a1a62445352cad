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
