"""CPU: the table-function host (csrc/host/cudasp_host.cpp) under
ThreadSanitizer and AddressSanitizer + UndefinedBehaviorSanitizer.

The host is the concurrent part of the library: executor threads reserve,
copy, publish and harvest batch slots of shared device feeds under one lock
per feed, reuse slots out of order, open them in a ring bound, and emit from
the last thread.  Its null-device mode (CUDASP_TF_NULL_DEVICE: feeds of plain
host memory, every slot done at launch, no device call) runs all of that
without a GPU, so the host is compiled here with the sanitizers (host code
only: -Xarch_host), linked ahead of the in-tree library (whose own host
symbols it interposes), and driven by tools/host_e2e --null-device
--cpu-table: many threads, 1 and 8 feeds, row chunks and Arrow columns,
small batches (many slot cycles), fixed and variable output lists.  The C
pinned table (csrc/host/pinned_table.cpp) is compiled in the same way and its
appends run under them too (host_e2e --pinned --null-device: batches in plain
host memory, runs spanning batches, 1 to 4 logical GPUs).  Any sanitizer
report fails the test."""
import json
import os
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "duckdb-cudasp-extension_amd")
HIPCC = "/opt/rocm/bin/hipcc"

SANITIZERS = {
    "thread": ["-fsanitize=thread"],
    "address,undefined": ["-fsanitize=address", "-fsanitize=undefined", "-fno-sanitize-recover=undefined"],
}


@pytest.fixture(scope="module", params=sorted(SANITIZERS), ids=lambda s: s.replace(",", "+"))
def sanitized(request):
    lib = os.path.join(PKG, "libcudasp_amd.so")
    if not os.path.exists(lib):
        pytest.fail("build the library first (make -C duckdb-cudasp-extension_amd)")
    flags = []
    for f in SANITIZERS[request.param]:
        flags += ["-Xarch_host", f]
    d = tempfile.mkdtemp(prefix="cudasp_san_")
    common = [HIPCC, "-O1", "-g", "-std=c++17", "--offload-arch=gfx950", "-fno-omit-frame-pointer"] + flags
    subprocess.check_call(common + ["-fPIC", "-c", "-o", os.path.join(d, "host.o"),
                                    os.path.join(PKG, "csrc", "host", "cudasp_host.cpp")])
    subprocess.check_call(common + ["-fPIC", "-c", "-o", os.path.join(d, "pinned.o"),
                                    os.path.join(PKG, "csrc", "host", "pinned_table.cpp")])
    subprocess.check_call(common + ["-c", "-o", os.path.join(d, "e2e.o"), os.path.join(ROOT, "tools", "host_e2e.cpp")])
    exe = os.path.join(d, "host_e2e")
    subprocess.check_call([HIPCC, "--offload-arch=gfx950"] + flags + ["-o", exe, os.path.join(d, "e2e.o"),
                                                                       os.path.join(d, "host.o"),
                                                                       os.path.join(d, "pinned.o"), "-L" + PKG,
                                                                       "-lcudasp_amd", "-Wl,-rpath," + PKG, "-lpthread"])
    # the sanitized host is the one that runs: the executable defines the
    # host's entry points (interposing the library's) and the sanitizer runtime
    syms = subprocess.check_output(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-s", "--wide", exe], text=True)
    defined = {ln.split()[-1] for ln in syms.splitlines() if len(ln.split()) >= 8 and ln.split()[6] != "UND"}
    assert "cudasp_tf_function" in defined and "cudasp_tf_init" in defined and "cudasp_pinned_append" in defined
    assert ("__tsan_init" if request.param == "thread" else "__asan_init") in defined
    return request.param, exe


CASES = [
    # device map, threads, batch_size, input, outputs
    ("0", 12, 2048, "rows", ["--outputs-max", "7"]),
    (",".join(["0"] * 8), 16, 4096, "columns", ["--outputs", "2"]),
    ("0,0,0", 6, 20000, "rows", ["--outputs", "2"]),
    ("0,0", 8, 4096, "vectors", ["--outputs-max", "5"]),
]


@pytest.mark.parametrize("case", CASES, ids=["1feed-rows", "8feeds-columns", "3feeds-rows", "2feeds-vectors"])
def test_host_feeds_clean_under_sanitizers(sanitized, case):
    name, exe = sanitized
    dmap, threads, batch, inp, outs = case
    env = dict(os.environ, CUDASP_TF_DEVICE_MAP=dmap, TSAN_OPTIONS="halt_on_error=1:report_signal_unsafe=0",
               ASAN_OPTIONS="detect_leaks=0:halt_on_error=1", UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([exe, "--null-device", "--cpu-table", "--rows", "150000", "--threads", str(threads), "--batch",
                        str(batch), "--input", inp, "--reps", "2"] + outs, capture_output=True, text=True,
                       timeout=600, env=env)
    assert "Sanitizer" not in r.stderr and "runtime error" not in r.stderr, (name, r.stderr[-4000:])
    assert r.returncode == 0, (name, r.returncode, r.stderr[-2000:])
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["null_device"] is True and res["emitted_equal_planted"] is True  # null device: nothing emitted
    assert res["feeds"] == len(dmap.split(","))
    assert res["launches"] >= 150000 // batch


@pytest.mark.parametrize("devices,batch,outs", [("0", 4096, ["--outputs-max", "7"]), ("0,0,0,0", 70000, ["--outputs", "2"])])
def test_pinned_appends_clean_under_sanitizers(sanitized, devices, batch, outs):
    name, exe = sanitized
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1:report_signal_unsafe=0",
               ASAN_OPTIONS="detect_leaks=0:halt_on_error=1", UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([exe, "--null-device", "--cpu-table", "--rows", "150000", "--batch", str(batch),
                        "--pinned", devices] + outs, capture_output=True, text=True, timeout=600, env=env)
    assert "Sanitizer" not in r.stderr and "runtime error" not in r.stderr, (name, r.stderr[-4000:])
    assert r.returncode == 0, (name, r.returncode, r.stderr[-2000:])
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["null_device"] is True and res["rows_pinned"] == 150000
    assert res["batches"] == -(-150000 // batch) and res["devices"] == [int(x) for x in devices.split(",")]
