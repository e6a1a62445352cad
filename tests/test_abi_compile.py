"""CPU: the reference host's own forward declarations of the kernel ABI
compile against include/cudasp_abi.h and link against libcudasp_amd.so.

The reference host declares LaunchBatchScan / RunBatchScanKernels /
FreeBatchScanState itself (/root/reference/src/cudasp_extension.cu:20-52).
This test extracts that `extern "C"` block from the reference AT TEST TIME
(no reference text is committed), compiles it in one C++ translation unit
after `#include "cudasp_abi.h"` -- a C-linkage redeclaration whose parameter
or return types differ is a hard error -- and links a program that takes the
address of each function against the in-tree library, so the reference host
would link unchanged.  Skipped where /root/reference is absent (the GPU box)."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference/src/cudasp_extension.cu"
LIB_DIR = os.path.join(ROOT, "duckdb-cudasp-extension_amd")

pytestmark = pytest.mark.skipif(not os.path.exists(REF), reason="reference sources absent")


def _extern_block():
    src = open(REF).read()
    m = re.search(r'extern\s+"C"\s*\{', src)
    assert m, "no extern \"C\" block in the reference host"
    depth, i = 1, m.end()
    while depth:
        c = src[i]
        depth += c == "{"
        depth -= c == "}"
        i += 1
    block = src[m.start():i]
    for name in ("LaunchBatchScan", "RunBatchScanKernels", "FreeBatchScanState"):
        assert name in block
    return block


def _compile(tmp_path, block, extra=""):
    tu = tmp_path / "ref_decls.cpp"
    tu.write_text('#include <cstddef>\n#include <cstdint>\n#include "cudasp_abi.h"\n' + block + "\n" + extra + """
int main() {
  void* fns[] = {(void*)&LaunchBatchScan, (void*)&RunBatchScanKernels, (void*)&FreeBatchScanState};
  return fns[0] && fns[1] && fns[2] ? 0 : 1;
}
""")
    cxx = shutil.which("g++") or shutil.which("c++")
    cmd = [cxx, "-std=c++17", "-Werror", "-I", os.path.join(ROOT, "include"), str(tu), "-o", str(tmp_path / "a.out"),
           "-L", LIB_DIR, "-lcudasp_amd", "-Wl,--allow-shlib-undefined"]
    return subprocess.run(cmd, capture_output=True, text=True)


def test_reference_declarations_compile_and_link(tmp_path):
    if not os.path.exists(os.path.join(LIB_DIR, "libcudasp_amd.so")):
        pytest.skip("libcudasp_amd.so not built")
    r = _compile(tmp_path, _extern_block())
    assert r.returncode == 0, r.stderr


def test_a_mismatched_declaration_is_rejected(tmp_path):
    """Control: the same check fails for a declaration whose type differs
    (count as uint64_t), so a passing test means the types agree."""
    block = _extern_block().replace("uint32_t count,\n", "uint64_t count,\n", 1)
    assert "uint64_t count" in block
    r = _compile(tmp_path, block)
    assert r.returncode != 0
    assert "conflicting" in r.stderr or "error" in r.stderr
