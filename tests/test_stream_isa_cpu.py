"""CPU: the streaming kernel's host/device ordering, checked in the gfx950
code object the library ships (no GPU needed).

k_scan_stream's correctness across PCIe and the 8 XCDs rests on the exact
stores the compiler emits (csrc/scan_kernels.hip, stream_poll and
stream_emit), not only on the HIP memory model:

* the poller mirrors a descriptor as a seqlock write -- seq invalidated,
  the fields, then seq -- every store an agent-scope write-through
  `global_store_dwordx2 ... sc1` (no sc0), each step separated from the
  next by `s_waitcnt vmcnt(0)` (it relies on those waits, not on release
  fences, which on gfx950 are whole-L2 write-backs), and the mirrored counts
  (pub_wr, pub) stored only after a further vmcnt(0);
* the wave that completes a batch stores its match count, then a
  system-scope release (`buffer_wbl2 sc0 sc1`), a vmcnt(0), and only then
  the done word, as a system-scope store (`sc0 sc1`).

A compiler or target change that reorders or drops any of these fails here.
The structure offsets come from the same headers (tests/native emu build).
"""
import ctypes
import os
import re
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "duckdb-cudasp-extension_amd", "libcudasp_amd.so")
EMU = os.path.join(ROOT, "tests", "native", "libcudasp_emu29.so")
LLVM = "/opt/rocm/lib/llvm/bin"
KERNELS = ("_Z13k_scan_streamILi26ELb0E", "_Z13k_scan_streamILi22ELb0E", "_Z13k_scan_streamILi26ELb1E",
           "_Z13k_scan_streamILi22ELb1E")


def layout():
    lib = ctypes.CDLL(EMU)
    out = (ctypes.c_uint64 * 8)()
    assert lib.emu_stream_layout(out, 8) == 8
    keys = ("ctrl_done", "ctrl_nmatch", "ctrl_desc", "batch_size", "batch_seq", "dev_desc", "dev_pub_wr", "dev_pub")
    return dict(zip(keys, [int(v) for v in out]))


@pytest.fixture(scope="module")
def disasm():
    """The library's gfx950 code object, disassembled: {kernel: [lines]}."""
    assert os.path.exists(LIB), "build the library first (make -C duckdb-cudasp-extension_amd)"
    with tempfile.TemporaryDirectory() as d:
        fat, co = os.path.join(d, "fatbin"), os.path.join(d, "co.o")
        subprocess.check_call([os.path.join(LLVM, "llvm-objcopy"), "--dump-section=.hip_fatbin=" + fat, LIB,
                               os.path.join(d, "stripped")])
        targets = subprocess.check_output([os.path.join(LLVM, "clang-offload-bundler"), "--list", "--type=o",
                                           "--input=" + fat], text=True).split()
        gfx = [t for t in targets if t.startswith("hip")]
        assert gfx == ["hipv4-amdgcn-amd-amdhsa--gfx950"], targets  # one device target: gfx950
        subprocess.check_call([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o",
                               "--targets=" + gfx[0], "--input=" + fat, "--output=" + co])
        text = subprocess.check_output([os.path.join(LLVM, "llvm-objdump"), "-d", "--mcpu=gfx950", co], text=True)
    kernels, cur = {}, None
    for line in text.splitlines():
        m = re.match(r"^[0-9a-f]+ <(\S+)>:", line)
        if m:
            cur = m.group(1)
            kernels[cur] = []
        elif cur and line.startswith("\t"):
            kernels[cur].append(line.split("//")[0].strip())
    return kernels


def kernel(disasm, prefix):
    names = [k for k in disasm if k.startswith(prefix)]
    assert len(names) == 1, (prefix, names)
    return disasm[names[0]]


def is_store(ins):
    return re.match(r"(global|flat|buffer)_store_|(global|flat|buffer)_atomic_", ins) is not None


def offset(ins):
    m = re.search(r"offset:(\d+)", ins)
    return int(m.group(1)) if m else 0


def cpol(ins):
    return set(re.findall(r"\b(sc0|sc1|nt)\b", ins))


def check_poller(code, L):
    seq_off = L["dev_desc"] + L["batch_seq"]
    field_offs = [L["dev_desc"] + 8 * i for i in range(L["batch_seq"] // 8)]
    seq_stores = [i for i, ins in enumerate(code) if ins.startswith("global_store_dwordx2") and offset(ins) == seq_off]
    assert len(seq_stores) >= 2, "no seqlock stores of the descriptor's seq found"
    checked = 0
    for a, b in zip(seq_stores, seq_stores[1:]):
        between = code[a + 1:b]
        stores = [(j, ins) for j, ins in enumerate(between) if is_store(ins)]
        if [offset(ins) for _, ins in stores] != field_offs:
            continue  # not an invalidate -> fields -> seq run
        for ins in [code[a], code[b]] + [ins for _, ins in stores]:
            assert ins.startswith("global_store_dwordx2"), ins
            assert cpol(ins) == {"sc1"}, "descriptor store not agent-scope write-through: " + ins
        first, last = stores[0][0], stores[-1][0]
        assert "s_waitcnt vmcnt(0)" in between[:first], "seq invalidation not complete before the fields"
        assert "s_waitcnt vmcnt(0)" in between[last + 1:], "fields not complete before seq is set"
        # the mirrored counts follow the descriptors, behind another vmcnt(0)
        after = code[b + 1:b + 40]
        pub_wr = [j for j, ins in enumerate(after) if is_store(ins) and offset(ins) == L["dev_pub_wr"]]
        pub = [j for j, ins in enumerate(after) if is_store(ins) and offset(ins) == L["dev_pub"]]
        assert pub_wr and pub and pub_wr[0] < pub[0], "pub_wr / pub stores not found after the descriptor"
        assert "s_waitcnt vmcnt(0)" in after[:pub_wr[0]], "counts stored before the descriptor completed"
        for j in (pub_wr[0], pub[0]):
            assert cpol(after[j]) == {"sc1"}, after[j]
        checked += 1
    assert checked == 1, "expected exactly one poller mirror sequence, found %d" % checked


def check_done(code, L):
    done = range(L["ctrl_done"], L["ctrl_done"] + 4 * 64)
    nmatch = range(L["ctrl_nmatch"], L["ctrl_nmatch"] + 4 * 64)
    done_stores = [i for i, ins in enumerate(code)
                   if ins.startswith("global_store_dword ") and offset(ins) in done and cpol(ins) >= {"sc0", "sc1"}]
    assert done_stores, "no system-scope store to the done words found"
    for i in done_stores:
        k = max(j for j in range(i) if code[j].startswith("buffer_wbl2") or is_store(code[j]))
        assert code[k] == "buffer_wbl2 sc0 sc1", "done word not directly behind a system-scope release: %s" % code[k]
        assert "s_waitcnt vmcnt(0)" in code[k + 1:i], "release not complete before the done word"
        prev = max(j for j in range(k) if is_store(code[j]))
        assert offset(code[prev]) in nmatch and cpol(code[prev]) >= {"sc0", "sc1"}, \
            "the match count is not the store released before the done word: " + code[prev]


@pytest.mark.parametrize("prefix", KERNELS)
def test_poller_descriptor_stores_are_ordered_write_through(disasm, prefix):
    check_poller(kernel(disasm, prefix), layout())


@pytest.mark.parametrize("prefix", KERNELS)
def test_done_word_follows_system_release(disasm, prefix):
    check_done(kernel(disasm, prefix), layout())


def check_prefetch_acquire(code):
    """The piece prefetch's system-scope acquire: one `buffer_inv sc0 sc1` in
    the kernel, with the piece's 16-byte loads of the row blobs after it."""
    inv = [i for i, ins in enumerate(code) if ins == "buffer_inv sc0 sc1"]
    assert len(inv) == 1, inv
    assert any(re.match(r"(global|flat)_load_dwordx4", ins) for ins in code[inv[0]:inv[0] + 800]), "no blob loads after it"


@pytest.mark.parametrize("prefix", KERNELS)
def test_piece_prefetch_acquires_host_memory(disasm, prefix):
    """Before a piece's reads of the pinned slots, a system-scope acquire: a
    slot rewritten by the host for a newer batch must not be read from lines
    the GPU still caches (the stale reads lost matches with 4 slots;
    test_host_stream_slot_reuse_reads_fresh_rows)."""
    check_prefetch_acquire(kernel(disasm, prefix))


def test_checks_reject_reordered_code(disasm):
    """Controls: the same code with one wait, fence or cache-policy bit
    removed fails the checks."""
    L = layout()
    code = kernel(disasm, KERNELS[0])
    seq_off = L["dev_desc"] + L["batch_seq"]
    last_seq = max(i for i, ins in enumerate(code) if ins.startswith("global_store_dwordx2") and offset(ins) == seq_off)
    wait = max(i for i in range(last_seq) if code[i] == "s_waitcnt vmcnt(0)")
    no_wait = code[:wait] + [c for c in code[wait:last_seq] if c != "s_waitcnt vmcnt(0)"] + code[last_seq:]
    with pytest.raises(AssertionError):
        check_poller(no_wait, L)
    no_sc1 = list(code)
    no_sc1[last_seq] = no_sc1[last_seq].replace(" sc1", "")
    with pytest.raises(AssertionError):
        check_poller(no_sc1, L)
    no_fence = [c for c in code if not c.startswith("buffer_wbl2")]
    with pytest.raises(AssertionError):
        check_done(no_fence, L)
    no_acquire = [c for c in code if c != "buffer_inv sc0 sc1"]
    with pytest.raises(AssertionError):
        check_prefetch_acquire(no_acquire)


def test_device_code_is_gfx950_only():
    """scan_stream.hpp refuses any other offload target at compile time."""
    src = os.path.join(ROOT, "duckdb-cudasp-extension_amd", "csrc", "scan_stream.hpp")
    text = open(src).read()
    assert "#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)" in text and "#error" in text
