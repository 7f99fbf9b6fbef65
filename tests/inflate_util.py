"""Shared helpers of the BGZF inflate tests: raw-DEFLATE members laid out as in a BGZF file, sample payloads, a
BGZF member walk, and calls of spg_bgzf_inflate (GPU) / spg_bgzf_inflate_check (the same decoder on the host)."""
import ctypes as C
import zlib

import numpy as np


class Member(C.Structure):
    _fields_ = [("coff", C.c_uint64), ("clen", C.c_uint32), ("ulen", C.c_uint32), ("uoff", C.c_uint64)]


def inflate(comp: bytes, members, gpu=True):
    from covid_spings_variant_caller_amd import _native as N
    L = N.gpu_lib()
    arr = (Member * max(1, len(members)))(*[Member(*m) for m in members])
    total = sum(m[2] for m in members)
    out = np.zeros(total + 16, np.uint8)
    st = np.full(max(1, len(members)), 99, np.uint32)
    cbuf = np.frombuffer(comp, np.uint8)
    ms = C.c_float(0)
    if gpu:
        rc = L.spg_bgzf_inflate(0, cbuf.ctypes.data, len(comp), C.addressof(arr), len(members), out.ctypes.data, total,
                                st.ctypes.data, C.byref(ms))
    else:
        rc = L.spg_bgzf_inflate_check(cbuf.ctypes.data, len(comp), C.addressof(arr), len(members), out.ctypes.data, total,
                                      st.ctypes.data)
    assert rc == 0, L.spg_bgzf_last_error()
    return out[:total].tobytes(), st[:len(members)], ms.value


def inflate_par_host(comp: bytes, members):
    """spg_bgzf_inflate_par_check: the parallel inflater's algorithm run on the host (status 0 or 100 = left to the
    lane-per-member decoder), and its stats (include/spings_gpu.h)."""
    from covid_spings_variant_caller_amd import _native as N
    L = N.gpu_lib()
    arr = (Member * max(1, len(members)))(*[Member(*m) for m in members])
    total = sum(m[2] for m in members)
    out = np.zeros(total + 16, np.uint8)
    st = np.full(max(1, len(members)), 99, np.uint32)
    stats = np.zeros(10, np.uint64)
    cbuf = np.frombuffer(comp, np.uint8)
    rc = L.spg_bgzf_inflate_par_check(cbuf.ctypes.data, len(comp), C.addressof(arr), len(members), out.ctypes.data,
                                      total, st.ctypes.data, stats.ctypes.data)
    assert rc == 0, L.spg_bgzf_last_error()
    return out[:total].tobytes(), st[:len(members)], stats


def fallbacks(device=0):
    """members of the last spg_bgzf_inflate that the parallel kernel left to the lane-per-member decoder"""
    from covid_spings_variant_caller_amd import _native as N
    n = C.c_int64(-1)
    assert N.gpu_lib().spg_bgzf_fallbacks(device, C.byref(n)) == 0
    return n.value


def pack(payloads):
    """members laid out as in a BGZF file: payload then an 8-byte trailer (CRC32, ISIZE)."""
    comp, members, uoff = bytearray(), [], 0
    for raw, data in payloads:
        coff = len(comp)
        comp += raw
        comp += zlib.crc32(data).to_bytes(4, "little") + len(data).to_bytes(4, "little")
        members.append((coff, len(raw), len(data), uoff))
        uoff += len(data)
    return bytes(comp), members


def deflate(data, level, strategy):
    c = zlib.compressobj(level, zlib.DEFLATED, -15, 9, strategy)
    return c.compress(data) + c.flush()


def samples(rng):
    quals = rng.choice(np.arange(2, 42, dtype=np.uint8), size=60000).tobytes()
    bam_like = bytes(rng.integers(0, 16, 30000, dtype=np.uint8)) + quals[:30000]
    text = (b"the quick brown fox jumps over the lazy dog " * 1500)[:65536]
    rnd = rng.integers(0, 256, 65536, dtype=np.uint8).tobytes()
    runs = bytes(np.repeat(rng.integers(0, 4, 4000, dtype=np.uint8), 16))
    return [quals, bam_like, text, rnd, runs, b"", b"a", b"ab" * 20000]


def all_block_types(rng):
    payloads = []
    for data in samples(rng):
        for level in (0, 1, 6, 9):
            for strategy in (zlib.Z_DEFAULT_STRATEGY, zlib.Z_FILTERED, zlib.Z_HUFFMAN_ONLY, zlib.Z_RLE, zlib.Z_FIXED):
                payloads.append((deflate(data, level, strategy), data))
    return payloads


def corrupt_set(rng):
    good = rng.choice(np.arange(2, 42, dtype=np.uint8), size=40000).tobytes()
    raw = deflate(good, 6, zlib.Z_DEFAULT_STRATEGY)
    bad = bytearray(raw)
    for i in range(20, len(bad), 97):
        bad[i] ^= 0x5A
    junk = rng.integers(0, 256, 3000, dtype=np.uint8).tobytes()
    return good, [(raw, good), (bytes(bad), good), (junk, good), (raw[:len(raw) // 2], good)]


def bgzf_members(raw: bytes):
    """(coff, clen, ulen, uoff) of every member of a BGZF file's bytes."""
    members, q, uoff = [], 0, 0
    while q < len(raw):
        xlen = int.from_bytes(raw[q + 10:q + 12], "little")
        x, bsize = q + 12, None
        while x < q + 12 + xlen:
            slen = int.from_bytes(raw[x + 2:x + 4], "little")
            if raw[x] == 66 and raw[x + 1] == 67:
                bsize = int.from_bytes(raw[x + 4:x + 6], "little") + 1
            x += 4 + slen
        isize = int.from_bytes(raw[q + bsize - 4:q + bsize], "little")
        members.append((q + 12 + xlen, bsize - xlen - 20, isize, uoff))
        uoff += isize
        q += bsize
    return members
