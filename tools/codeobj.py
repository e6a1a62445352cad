"""Identify the machine code a PMC summary was measured on.

The HIP library carries its gfx950 code object in a clang offload bundle
(`.hip_fatbin`).  `kernel_stamp(lib, pattern)` returns the SHA-256 of one
kernel's machine code (its function bytes plus its kernel descriptor), so a
summary under profiles/ can say exactly which kernel it counted, and bench.py
can refuse counters taken on a different build of that kernel.  Changes to the
host code or to other kernels leave the stamp unchanged.

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


def kernel_stamp(lib_path, pattern, arch="gfx950"):
    """SHA-256 (hex, first 16 bytes) of the machine code and descriptor of the
    one kernel whose mangled name matches `pattern` (re.search)."""
    rx = re.compile(pattern)
    for _, elf in code_objects(lib_path, arch):
        syms, secs = symbols(elf)
        hits = [n for n, (v, sz, t, sh) in syms.items() if t == 2 and rx.search(n)]  # STT_FUNC
        if len(hits) > 1:
            raise ValueError("pattern %r matches several kernels: %s" % (pattern, hits))
        if hits:
            name = hits[0]
            v, sz, _, sh = syms[name]
            h = hashlib.sha256(_bytes_at(elf, secs, sh, v, sz))
            kd = syms.get(name + ".kd")
            if kd:
                h.update(_bytes_at(elf, secs, kd[3], kd[0], kd[1]))
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
