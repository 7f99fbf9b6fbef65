"""BGZF members inflated on the GPU (spg_bgzf_inflate, csrc/spg_inflate.hip): every DEFLATE block type and zlib
strategy against Python's zlib, a simulated BAM's members against gzip, and corrupt members reported (never a fault).
The reference reads BAMs through pysam/htslib's BGZF reader (live_variant_caller.py:54-72); the bytes must be
identical."""
import ctypes as C
import gzip
import os
import zlib

import numpy as np
import pytest

import spings  # noqa: F401

pytestmark = pytest.mark.gpu


class Member(C.Structure):
    _fields_ = [("coff", C.c_uint64), ("clen", C.c_uint32), ("ulen", C.c_uint32), ("uoff", C.c_uint64)]


def _inflate(comp: bytes, members):
    from covid_spings_variant_caller_amd import _native as N
    L = N.gpu_lib()
    arr = (Member * max(1, len(members)))(*[Member(*m) for m in members])
    total = sum(m[2] for m in members)
    out = np.zeros(total + 16, np.uint8)
    st = np.full(max(1, len(members)), 99, np.uint32)
    cbuf = np.frombuffer(comp, np.uint8)
    ms = C.c_float(0)
    rc = L.spg_bgzf_inflate(0, cbuf.ctypes.data, len(comp), C.addressof(arr), len(members), out.ctypes.data, total,
                            st.ctypes.data, C.byref(ms))
    assert rc == 0, L.spg_bgzf_last_error()
    return out[:total].tobytes(), st[:len(members)], ms.value


def _pack(payloads):
    """members laid out as in a BGZF file: payload then an 8-byte trailer (CRC32, ISIZE)."""
    comp, members, uoff = bytearray(), [], 0
    for raw, data in payloads:
        coff = len(comp)
        comp += raw
        comp += zlib.crc32(data).to_bytes(4, "little") + len(data).to_bytes(4, "little")
        members.append((coff, len(raw), len(data), uoff))
        uoff += len(data)
    return bytes(comp), members


def _deflate(data, level, strategy):
    c = zlib.compressobj(level, zlib.DEFLATED, -15, 9, strategy)
    return c.compress(data) + c.flush()


def _samples(rng):
    quals = rng.choice(np.arange(2, 42, dtype=np.uint8), size=60000, p=None).tobytes()
    bam_like = bytes(rng.integers(0, 16, 30000, dtype=np.uint8)) + quals[:30000]
    text = (b"the quick brown fox jumps over the lazy dog " * 1500)[:65536]
    rnd = rng.integers(0, 256, 65536, dtype=np.uint8).tobytes()
    runs = bytes(np.repeat(rng.integers(0, 4, 4000, dtype=np.uint8), 16))
    return [quals, bam_like, text, rnd, runs, b"", b"a", b"ab" * 20000]


def test_every_block_type_and_strategy_matches_zlib():
    rng = np.random.default_rng(7)
    payloads = []
    for data in _samples(rng):
        for level in (0, 1, 6, 9):
            for strategy in (zlib.Z_DEFAULT_STRATEGY, zlib.Z_FILTERED, zlib.Z_HUFFMAN_ONLY, zlib.Z_RLE, zlib.Z_FIXED):
                payloads.append((_deflate(data, level, strategy), data))
    comp, members = _pack(payloads)
    out, st, _ = _inflate(comp, members)
    assert (st == 0).all(), [(i, int(s)) for i, s in enumerate(st) if s]
    assert out == b"".join(d for _, d in payloads)


def test_simulated_bam_members_match_gzip(tmp_path):
    from covid_spings_variant_caller_amd import synth
    from covid_spings_variant_caller_amd.pileup import simulate_bam
    ref = synth.reference(3000, seed=3)
    bam = str(tmp_path / "s.bam")
    simulate_bam(bam, "NC_045512.2", ref, depth=400.0, seed=5, n_threads=4)
    raw = open(bam, "rb").read()
    members, q, uoff = [], 0, 0
    while q < len(raw):
        xlen = int.from_bytes(raw[q + 10:q + 12], "little")
        x, bsize = q + 12, None
        while x < q + 12 + xlen:
            si1, si2, slen = raw[x], raw[x + 1], int.from_bytes(raw[x + 2:x + 4], "little")
            if si1 == 66 and si2 == 67:
                bsize = int.from_bytes(raw[x + 4:x + 6], "little") + 1
            x += 4 + slen
        isize = int.from_bytes(raw[q + bsize - 4:q + bsize], "little")
        members.append((q + 12 + xlen, bsize - xlen - 20, isize, uoff))
        uoff += isize
        q += bsize
    assert len(members) > 10
    out, st, _ = _inflate(raw, members)
    assert (st == 0).all()
    assert out == gzip.decompress(raw)


def test_corrupt_members_are_reported():
    rng = np.random.default_rng(9)
    good = rng.choice(np.arange(2, 42, dtype=np.uint8), size=40000).tobytes()
    raw = _deflate(good, 6, zlib.Z_DEFAULT_STRATEGY)
    bad = bytearray(raw)
    for i in range(20, len(bad), 97):
        bad[i] ^= 0x5A
    junk = rng.integers(0, 256, 3000, dtype=np.uint8).tobytes()
    comp, members = _pack([(raw, good), (bytes(bad), good), (junk, good), (raw[:len(raw) // 2], good)])
    out, st, _ = _inflate(comp, members)
    assert st[0] == 0 and out[:len(good)] == good
    assert (st[1:] != 0).all(), st
