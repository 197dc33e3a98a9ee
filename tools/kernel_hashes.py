"""Per-kernel code hashes of librsp.so's gfx950 code objects (bench provenance).

usage: kernel_hashes.py LIBRSP.so OUT.json

The HIP fat binary in the .so holds one clang offload bundle per device translation unit; its
gfx950 entry is an AMDGPU ELF.  For every kernel symbol (STT_FUNC with a `.kd` descriptor) the
bytes of its code are hashed; kernels are keyed by their short name (the identifier before the
template arguments, as tools/pmc_traffic.py keys its counters), all instantiations of a name
hashed together in mangled-name order.  bench.py compares these with the hashes a PMC traffic
file recorded when it was measured: a kernel whose code changed since has no measured traffic.
"""
import hashlib
import json
import re
import struct
import sys

MAGIC = b'__CLANG_OFFLOAD_BUNDLE__'


def code_objects(blob):
    i = blob.find(MAGIC)
    while i >= 0:
        n = struct.unpack_from('<Q', blob, i + 24)[0]
        p = i + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from('<QQQ', blob, p)
            triple = blob[p + 24:p + 24 + tl].decode()
            p += 24 + tl
            if 'amdgcn' in triple and size:
                yield triple, blob[i + off:i + off + size]
        i = blob.find(MAGIC, i + 1)


def kernel_code(elf):
    """{mangled kernel name: bytes of its code} from one AMDGPU ELF (64-bit little endian)."""
    assert elf[:4] == b'\x7fELF' and elf[4] == 2 and elf[5] == 1
    shoff, = struct.unpack_from('<Q', elf, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from('<HHH', elf, 0x3A)
    secs = [struct.unpack_from('<IIQQQQIIQQ', elf, shoff + k * shentsize) for k in range(shnum)]
    out = {}
    for s in secs:
        if s[1] != 2:   # SHT_SYMTAB
            continue
        strtab = secs[s[6]]
        for k in range(s[5] // s[9]):
            name_off, info, other, shndx, value, size = struct.unpack_from('<IBBHQQ', elf, s[4] + k * s[9])
            if info & 0xF != 2 or size == 0 or shndx >= len(secs):   # STT_FUNC with code
                continue
            nm = elf[strtab[4] + name_off:elf.index(b'\0', strtab[4] + name_off)].decode()
            sec = secs[shndx]
            out[nm] = elf[sec[4] + (value - sec[3]):sec[4] + (value - sec[3]) + size]
    return out


def short_name(mangled):
    """The kernel's identifier: the first source name of the mangled name that is not the
    anonymous namespace (`_ZN12_GLOBAL__N_110k1_dbf_mtdI...` -> k1_dbf_mtd)."""
    if not mangled.startswith('_Z'):
        return mangled
    p = 3 if mangled.startswith('_ZN') else 2
    while True:
        m = re.match(r'(\d+)', mangled[p:])
        if not m:
            return mangled
        n = int(m.group(1))
        name = mangled[p + len(m.group(1)):p + len(m.group(1)) + n]
        p += len(m.group(1)) + n
        if not name.startswith('_GLOBAL__N'):
            return name


def main():
    lib, out = sys.argv[1:3]
    blob = open(lib, 'rb').read()
    funcs = {}
    for _, elf in code_objects(blob):
        funcs.update(kernel_code(elf))
    kd = set()
    for _, elf in code_objects(blob):   # kernels = functions that have a kernel descriptor
        kd |= {n[:-3] for n in re.findall(rb'([_A-Za-z0-9]+\.kd)\0', elf) for n in [n.decode()]}
    groups = {}
    for nm in sorted(funcs):
        if nm in kd:
            groups.setdefault(short_name(nm), []).append(nm)
    res = {}
    for sn, names in sorted(groups.items()):
        h = hashlib.sha256()
        for nm in names:
            h.update(nm.encode() + b'\0' + funcs[nm])
        res[sn] = h.hexdigest()[:16]
    json.dump(res, open(out, 'w'), indent=1, sort_keys=True)


if __name__ == '__main__':
    main()
