"""Fingerprint of one kernel's machine code inside libsalp.so.

The library's device code is a clang offload bundle (section .hip_fatbin) per
translation unit, each holding a gfx950 ELF code object.  `kernel_sha(lib,
name)` hashes the bytes of the kernel's function symbol plus its kernel
descriptor (`<name>.kd`: register counts, LDS size), so the fingerprint moves
when that kernel's code or resources change and stays put when another
kernel of the library is edited.

PMC summaries (tools/pmc_summary.py) record the fingerprint of the kernel
they counted; bench.py reports their HBM traffic / fp64 mix only when the
fingerprint equals the one of the library it just ran.  Pure Python: no
ROCm tool is needed, so it works on the CPU container and on the GPU box.
"""
import hashlib
import struct

BUNDLE_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _code_objects(blob):
    """Every gfx9xx ELF code object of every offload bundle in `blob`."""
    pos = 0
    while True:
        b = blob.find(BUNDLE_MAGIC, pos)
        if b < 0:
            return
        pos = b + len(BUNDLE_MAGIC)
        (n,) = struct.unpack_from("<Q", blob, pos)
        p = pos + 8
        for _ in range(n):
            off, size, idlen = struct.unpack_from("<QQQ", blob, p)
            p += 24
            ident = blob[p:p + idlen].decode("ascii", "replace")
            p += idlen
            if "amdgcn" in ident and size > 0:
                co = blob[b + off:b + off + size]
                if co[:4] == b"\x7fELF":
                    yield ident, co


def _symbols(co):
    """{name: (file_offset, size)} of the code object's defined symbols."""
    shoff, = struct.unpack_from("<Q", co, 0x28)
    shentsize, shnum, _ = struct.unpack_from("<HHH", co, 0x3A)
    secs = []
    for k in range(shnum):
        (_name, sh_type, _flags, addr, off, size, link, _info, _align,
         entsize) = struct.unpack_from("<IIQQQQIIQQ", co, shoff + k * shentsize)
        secs.append((sh_type, addr, off, size, link, entsize))
    out = {}
    for sh_type, _addr, off, size, link, entsize in secs:
        if sh_type != 2:   # SHT_SYMTAB
            continue
        stroff = secs[link][2]
        for j in range(size // entsize):
            st_name, _st_info, _st_other, shndx, value, ssize = struct.unpack_from("<IBBHQQ", co, off + j * entsize)
            if shndx == 0 or shndx >= len(secs) or ssize == 0:
                continue
            end = co.index(b"\0", stroff + st_name)
            name = co[stroff + st_name:end].decode("ascii", "replace")
            s_addr, s_off = secs[shndx][1], secs[shndx][2]
            out[name] = (value - s_addr + s_off, ssize)
    return out


def kernel_symbols(lib_path, contains):
    """Names of the kernel symbols (with a .kd descriptor) whose name contains `contains`."""
    blob = open(lib_path, "rb").read()
    names = set()
    for _ident, co in _code_objects(blob):
        syms = _symbols(co)
        names |= {n for n in syms if contains in n and n + ".kd" in syms}
    return sorted(names)


def _mask_layout(code):
    """The kernel's machine code with the bytes that only say where things lie
    in the code object zeroed: the 32-bit literal of each `s_add_u32` /
    `s_addc_u32` that follows an `s_getpc_b64` (a PC-relative address of a
    global or a callee, which moves when anything else in the library grows or
    shrinks).  Everything else, branch offsets inside the kernel included, is
    kept."""
    n = len(code) // 4
    w = list(struct.unpack("<%dI" % n, code[:4 * n]))
    for i in range(n):
        if (w[i] & 0xFF80FFFF) != 0xBE801C00:       # s_getpc_b64 s[k:k+1]
            continue
        j = i + 1
        while j + 1 < n and j <= i + 4:
            op = w[j] & 0xFF800000
            lit = (w[j] & 0xFF) == 0xFF or (w[j] >> 8 & 0xFF) == 0xFF
            if op in (0x80000000, 0x82000000) and lit:   # s_add_u32 / s_addc_u32 with a literal
                w[j + 1] = 0
                j += 2
            else:
                j += 1
    return struct.pack("<%dI" % n, *w) + code[4 * n:]


def kernel_sha(lib_path, contains):
    """sha256 (hex, 16 chars) of the code + descriptor of the one kernel whose
    mangled name contains `contains`, or None (absent or ambiguous).  Layout
    bytes are masked (`_mask_layout`; the descriptor's
    kernel_code_entry_byte_offset, bytes 16-23), so the fingerprint changes
    with the kernel's own instructions, not with edits elsewhere in the
    library."""
    blob = open(lib_path, "rb").read()
    for _ident, co in _code_objects(blob):
        syms = _symbols(co)
        hits = [n for n in syms if contains in n and n + ".kd" in syms]
        if len(hits) == 1:
            symbol = hits[0]
            h = hashlib.sha256()
            off, size = syms[symbol]
            h.update(_mask_layout(co[off:off + size]))
            off, size = syms[symbol + ".kd"]
            kd = bytearray(co[off:off + size])
            kd[16:24] = bytes(8)
            h.update(bytes(kd))
            return h.hexdigest()[:16]
    return None


# The bench's dominant kernel: k_rollout<RAND = false, POL = false>.
ROLLOUT_KERNEL = "k_rolloutILb0ELb0EE"
# The PPO leg's collection kernel (config 5, 32 768 envs): the auto choice's
# two-wave kernel with POL = true -- k_rollout_split<true> from round 6
# (k_rollout_pair<true> with SALP_TWO_WAVE_KERNEL=pair).
PAIR_COLLECT_KERNEL = "k_rollout_pairILb1EE"
SPLIT_COLLECT_KERNEL = "k_rollout_splitILb1EE"


def collect_kernel():
    """(mangled-name fragment, display name) of the collection kernel the auto choice runs at config 5."""
    import os
    if (os.environ.get("SALP_TWO_WAVE_KERNEL") or "").startswith("p"):
        return PAIR_COLLECT_KERNEL, "k_rollout_pair<true>"
    return SPLIT_COLLECT_KERNEL, "k_rollout_split<true>"
