"""Identify the machine code a PMC summary was measured on.

The HIP library carries its gfx950 code object in a clang offload bundle
(`.hip_fatbin`).  `kernel_stamp(lib, pattern)` returns the SHA-256 of one
kernel's machine code -- its instructions with PC-relative address literals
resolved to the symbols they point at, plus its kernel descriptor -- so a
summary under profiles/ can say exactly which kernel it counted, and bench.py
can refuse counters taken on a different build of that kernel.  Changes to the
host code or to other kernels (which move this one in the code object) leave
the stamp unchanged.

  python tools/codeobj.py LIB [REGEX ...]   # list kernels / print stamps
"""
import hashlib
import re
import struct
import sys

BUNDLE_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _sections(elf):
    if elf[:4] != b"\x7fELF" or elf[4] != 2:
        raise ValueError("not an ELF64 object")
    shoff, = struct.unpack_from("<Q", elf, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", elf, 0x3A)
    secs = []
    for i in range(shnum):
        name, typ, flags, addr, off, size, link, info, align, entsize = struct.unpack_from(
            "<IIQQQQIIQQ", elf, shoff + i * shentsize)
        secs.append(dict(name_off=name, type=typ, addr=addr, off=off, size=size, link=link, entsize=entsize))
    strtab = secs[shstrndx]
    for s in secs:
        end = elf.index(b"\0", strtab["off"] + s["name_off"])
        s["name"] = elf[strtab["off"] + s["name_off"]:end].decode()
    return secs


def code_objects(lib_path, arch="gfx950"):
    """[(triple, bytes)] of the device code objects in the library's bundles."""
    data = open(lib_path, "rb").read()
    out = []
    pos = data.find(BUNDLE_MAGIC)
    while pos >= 0:
        n, = struct.unpack_from("<Q", data, pos + 24)
        p = pos + 32
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", data, p)
            triple = data[p + 24:p + 24 + tlen].decode()
            p += 24 + tlen
            if arch in triple and size:
                out.append((triple, data[pos + off:pos + off + size]))
        pos = data.find(BUNDLE_MAGIC, p)
    if not out:
        raise ValueError("no %s code object in %s" % (arch, lib_path))
    return out


def symbols(elf):
    """{name: (value, size, type)} of the code object's symbol table."""
    secs = _sections(elf)
    out = {}
    for s in secs:
        if s["type"] != 2:  # SHT_SYMTAB
            continue
        strs = secs[s["link"]]
        for i in range(s["size"] // 24):
            name, info, other, shndx, value, size = struct.unpack_from("<IBBHQQ", elf, s["off"] + i * 24)
            end = elf.index(b"\0", strs["off"] + name)
            nm = elf[strs["off"] + name:end].decode()
            if nm:
                out[nm] = (value, size, info & 0xF, shndx)
    return out, secs


def _bytes_at(elf, secs, shndx, value, size):
    sec = secs[shndx]
    start = sec["off"] + value - sec["addr"]
    return elf[start:start + size]


OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"


def _normalized_code(elf, secs, syms, name):
    """The kernel's instructions as text with every absolute address taken out:
    the disassembly without its address/encoding comments, and the literal of
    each PC-relative address computation (s_getpc_b64 + s_add_u32 /
    s_addc_u32) replaced by its target as `symbol+offset` (or `self+offset`).
    Independent of where the kernel and the globals it reads sit in the code
    object, so a change elsewhere in the library leaves it unchanged."""
    import subprocess
    import tempfile
    with tempfile.NamedTemporaryFile(suffix=".o") as f:
        f.write(elf)
        f.flush()
        out = subprocess.run([OBJDUMP, "-d", "--disassemble-symbols=" + name, f.name], capture_output=True,
                             text=True, check=True).stdout
    v0, size = syms[name][0], syms[name][1]
    objects = sorted((v, sz, n) for n, (v, sz, t, sh) in syms.items() if sz and n != name)

    def label(addr):
        if v0 <= addr < v0 + size:
            return "self+%d" % (addr - v0)
        for v, sz, n in objects:
            if v <= addr < v + sz:
                return "%s+%d" % (n, addr - v)
        return "?"

    lines = []
    pc = None  # (register pair low, address after s_getpc)
    for ln in out.splitlines():
        m = re.match(r"\s+(\w+)\s*(.*?)\s*//\s*([0-9A-Fa-f]+):", ln)
        if not m:
            continue
        op, args, addr = m.group(1), m.group(2), int(m.group(3), 16)
        if op == "s_getpc_b64":
            reg = re.match(r"s\[(\d+):", args)
            pc = (reg.group(1), addr + 4) if reg else None
        elif pc and op in ("s_add_u32", "s_addc_u32"):
            parts = [x.strip() for x in args.split(",")]
            if len(parts) == 3 and parts[2].startswith("0x"):
                if op == "s_add_u32":
                    pc = (pc[0], pc[1], int(parts[2], 16))
                    args = "%s, %s, <pcrel>" % (parts[0], parts[1])
                else:
                    lo = pc[2] if len(pc) > 2 else 0
                    target = (pc[1] + lo + (int(parts[2], 16) << 32)) & ((1 << 64) - 1)
                    args = "%s, %s, <%s>" % (parts[0], parts[1], label(target))
                    pc = None
        lines.append(op + " " + args)
    return "\n".join(lines)


def kernel_stamp(lib_path, pattern, arch="gfx950"):
    """SHA-256 (hex, first 16 bytes) of the one kernel whose mangled name
    matches `pattern` (re.search): its normalized instructions
    (_normalized_code) and its kernel descriptor minus the code entry offset."""
    rx = re.compile(pattern)
    for _, elf in code_objects(lib_path, arch):
        syms, secs = symbols(elf)
        hits = [n for n, (v, sz, t, sh) in syms.items() if t == 2 and rx.search(n)]  # STT_FUNC
        if len(hits) > 1:
            raise ValueError("pattern %r matches several kernels: %s" % (pattern, hits))
        if hits:
            name = hits[0]
            v, sz, _, sh = syms[name]
            h = hashlib.sha256(_normalized_code(elf, secs, syms, name).encode())
            kd = syms.get(name + ".kd")
            if kd:
                d = bytearray(_bytes_at(elf, secs, kd[3], kd[0], kd[1]))
                d[16:24] = bytes(8)  # kernel_code_entry_byte_offset: where the code sits
                h.update(bytes(d))
            return dict(symbol=name, sha256=h.hexdigest()[:32], code_bytes=sz)
    raise ValueError("no kernel matching %r in %s" % (pattern, lib_path))


# kernels whose counters bench.py reads (mangled-name patterns)
K_SCAN_MULTI_26 = r"^_Z12k_scan_multiILi26ELb1EE"
K_LAYOUT_PROBE = r"^_Z14k_layout_probe"


def multi_pattern(fb_bits, pipelined=True):
    """k_scan_multi<fb_bits, pipelined>: the bench's timed kernel."""
    return r"^_Z12k_scan_multiILi%dELb%dEE" % (fb_bits, 1 if pipelined else 0)


def main():
    lib = sys.argv[1]
    pats = sys.argv[2:]
    if not pats:
        for _, elf in code_objects(lib):
            syms, _ = symbols(elf)
            for n, (v, sz, t, sh) in sorted(syms.items()):
                if t == 2:
                    print(sz, n)
        return
    for p in pats:
        print(kernel_stamp(lib, p))


if __name__ == "__main__":
    main()
