"""Incremental checkpoint manifest (live_variant_caller._read_manifest; create_checkpoint writes it): recognised
only for the manifest layout, None for absent, foreign, single-file-layout or pickled files (CPU; the GPU round
trips are in tests/test_live_caller_gpu.py)."""
import pickle

import numpy as np

import spings  # noqa: F401
from covid_spings_variant_caller_amd.live_variant_caller import _read_manifest


def test_manifest_roundtrip(tmp_path):
    f = str(tmp_path / "ck.npz")
    with open(f, "wb") as fh:
        np.savez(fh, format=np.int64(2), token=np.array("abc123"), contig=np.array([0, 0, 1], np.int64),
                 names=np.array(["chrA", "chrB"]), min_base_quality=np.int64(30),
                 shard_files=np.array(["ck.npz.abc.0.npz", "ck.npz.abc.2.npz"]),
                 shard_ranges=np.array([[0, 2], [2, 1]], np.int64))
    m = _read_manifest(f)
    assert m == {"token": "abc123", "names": ["chrA", "chrB"], "contig": [0, 0, 1], "n": 3,
                 "min_base_quality": 30, "shards": [("ck.npz.abc.0.npz", 0, 2), ("ck.npz.abc.2.npz", 2, 1)]}


def test_not_a_manifest(tmp_path):
    assert _read_manifest(str(tmp_path / "absent.npz")) is None
    old = str(tmp_path / "v1.npz")
    with open(old, "wb") as fh:
        np.savez(fh, contig=np.array([0], np.int64), names=np.array(["chrA"]), min_base_quality=np.int64(30),
                 b0_pos=np.int64(0), b0_off=np.zeros(2, np.uint64), b0_codes=np.zeros(0, np.uint8),
                 b0_quals=np.zeros(0, np.uint8))
    assert _read_manifest(old) is None
    txt = tmp_path / "t.npz"
    txt.write_text("not numpy")
    assert _read_manifest(str(txt)) is None
    pk = tmp_path / "p.npz"
    pk.write_bytes(pickle.dumps({"memory": {}}))      # the reference's pickle: never unpickled
    assert _read_manifest(str(pk)) is None


def test_shard_roundtrip_and_refusals(tmp_path):
    """The raw checkpoint shard (live_variant_caller._write_shard / _read_shard): batches written as they come read back
    identical; a file that is not a shard, a truncated one, or one naming another dtype is refused."""
    from covid_spings_variant_caller_amd.live_variant_caller import _read_shard, _write_shard
    rng = np.random.default_rng(3)
    batches = []
    for k in range(4):
        n = int(rng.integers(0, 50))
        lens = rng.integers(0, 9, n)
        off = np.zeros(n + 1, np.uint64)
        np.cumsum(lens, out=off[1:])
        batches.append((int(rng.integers(0, 1000)), off, rng.integers(0, 18, int(off[-1]), dtype=np.uint8),
                        rng.integers(0, 60, int(off[-1]), dtype=np.uint8)))
    p = str(tmp_path / "a.spgck")
    size = _write_shard(p, iter(batches))
    assert size == (tmp_path / "a.spgck").stat().st_size
    got = _read_shard(p)
    assert len(got) == len(batches)
    for (pa, oa, ca, qa), (pb, ob, cb, qb) in zip(got, batches):
        assert pa == pb and oa.dtype == np.uint64
        np.testing.assert_array_equal(oa, ob)
        np.testing.assert_array_equal(ca, cb)
        np.testing.assert_array_equal(qa, qb)
    import pytest
    bad = tmp_path / "b.spgck"
    bad.write_bytes(b"not a shard at all, just bytes")
    with pytest.raises(ValueError):
        _read_shard(str(bad))
    raw = (tmp_path / "a.spgck").read_bytes()
    (tmp_path / "t.spgck").write_bytes(raw[:-5])
    with pytest.raises(ValueError):
        _read_shard(str(tmp_path / "t.spgck"))
    (tmp_path / "d.spgck").write_bytes(raw.replace(b'"<u8"', b'"|O8"'))
    with pytest.raises(ValueError):
        _read_shard(str(tmp_path / "d.spgck"))


def test_packed_shard_roundtrip(tmp_path):
    """The packed batch form (engine.iter_history_packed / spg_history_copy_packed): one byte per kept entry —
    A/C/G/T (BAM nibbles 1/2/4/8) in the top 2 bits over q 0..62 — and an exception list for everything else
    (other codes, D / N entries 16 / 17, q >= 63), decoded on read; mixed with an unpacked batch in one shard."""
    import numpy as np
    from covid_spings_variant_caller_amd import live_variant_caller as LV
    rng = np.random.default_rng(5)
    codes = rng.choice(np.array([1, 2, 4, 8, 15, 16, 17, 3], np.uint8), size=5000, p=[.24, .24, .24, .24, .01, .01, .01, .01])
    quals = rng.integers(0, 94, 5000).astype(np.uint8)
    b2 = np.full(5000, 4, np.uint8)
    for k, c in enumerate((1, 2, 4, 8)):
        b2[codes == c] = k
    esc = (b2 == 4) | (quals >= 63)
    packed = np.where(esc, 63, (b2 << 6) | quals).astype(np.uint8)
    xi = np.nonzero(esc)[0].astype(np.uint64)
    perm = rng.permutation(len(xi))                      # (exceptions come in no particular order)
    ent = {"pos": 100, "off": np.array([0, 2000, 5000], np.uint64), "packed": packed, "xi": xi[perm],
           "xc": codes[esc][perm], "xq": quals[esc][perm]}
    plain = (7, np.array([0, 3], np.uint64), np.array([1, 16, 2], np.uint8), np.array([40, 0, 99], np.uint8))
    path = str(tmp_path / "s.spgck")
    LV._write_shard(path, [ent, plain])
    got = LV._read_shard(path)
    assert got[0][0] == 100 and (got[0][1] == ent["off"]).all()
    assert (got[0][2] == codes).all() and (got[0][3] == quals).all()
    assert got[1][0] == 7 and (got[1][2] == plain[2]).all() and (got[1][3] == plain[3]).all()


def test_shard_split_arrays_roundtrip(tmp_path, monkeypatch):
    """Large arrays go out in pieces written at once (the shard file and side files <shard>.x<j>): read back identical
    for ragged sizes (a piece may be empty), the byte count covers every file, a missing or short side file and a side
    name outside the shard's are refused, and _remove_unlisted deletes a shard's side files with it."""
    import os
    import pytest
    from covid_spings_variant_caller_amd import live_variant_caller as LV
    monkeypatch.setattr(LV, "_SHARD_SPLIT", 1000)
    rng = np.random.default_rng(11)
    batches = []
    for n_ent in (999, 1000, 4097, 12289, 3 * 4096 + 1):
        off = np.array([0, n_ent // 2, n_ent], np.uint64)
        batches.append((int(rng.integers(0, 100)), off, rng.integers(0, 18, n_ent, dtype=np.uint8),
                        rng.integers(0, 60, n_ent, dtype=np.uint8)))
    p = str(tmp_path / "spgck-t-0-5.spgck")
    size = LV._write_shard(p, batches)
    files = sorted(x for x in os.listdir(tmp_path) if x.startswith("spgck-t-0-5.spgck"))
    assert len(files) > 1 and not any(x.endswith(".tmp") for x in files)
    assert size == sum((tmp_path / x).stat().st_size for x in files)
    got = LV._read_shard(p)
    for (pa, oa, ca, qa), (pb, ob, cb, qb) in zip(got, batches):
        assert pa == pb
        np.testing.assert_array_equal(oa, ob)
        np.testing.assert_array_equal(ca, cb)
        np.testing.assert_array_equal(qa, qb)
    side = max((tmp_path / x for x in files[1:]), key=lambda q: q.stat().st_size)
    data = side.read_bytes()
    side.write_bytes(data[:-1])
    with pytest.raises(ValueError):
        LV._read_shard(p)
    side.unlink()
    with pytest.raises(OSError):
        LV._read_shard(p)
    raw = (tmp_path / "spgck-t-0-5.spgck").read_bytes()
    (tmp_path / "spgck-t-0-5.spgck").write_bytes(raw.replace(b"spgck-t-0-5.spgck.x", b"../../../etc/x"))
    with pytest.raises(ValueError):
        LV._read_shard(p)
    LV._remove_unlisted(str(tmp_path), {"spgck-t-0-5.spgck"})
    assert not [x for x in os.listdir(tmp_path) if x.startswith("spgck-t-0-5.spgck")]


def test_shard_split_reused_buffer_generator(tmp_path, monkeypatch):
    """engine.iter_history_packed yields views of ONE pinned staging buffer that its next batch
    overwrites.  Side-file pieces of a batch must be on disk before the generator is resumed: a generator that reuses
    one buffer over 3 batches (side writers slowed down) reads back every batch's own bytes."""
    import threading
    import time
    from covid_spings_variant_caller_amd import live_variant_caller as LV
    monkeypatch.setattr(LV, "_SHARD_SPLIT", 1000)
    orig = LV._shard_side

    def slow_side(path, j):
        if threading.current_thread() is not threading.main_thread():
            time.sleep(0.05)                          # (a helper thread still writing when the next batch arrives)
        return orig(path, j)

    monkeypatch.setattr(LV, "_shard_side", slow_side)
    n = 20000
    staging = np.zeros(2 * n, np.uint8)
    expect = []

    def gen():
        rng = np.random.default_rng(17)
        for k in range(3):
            codes = staging[:n]
            quals = staging[n:]
            codes[:] = rng.integers(0, 18, n, dtype=np.uint8)
            quals[:] = rng.integers(0, 60, n, dtype=np.uint8)
            expect.append((k, codes.copy(), quals.copy()))
            yield (k, np.array([0, n // 3, n], np.uint64), codes, quals)

    p = str(tmp_path / "spgck-r-0-3.spgck")
    LV._write_shard(p, gen())
    got = LV._read_shard(p)
    assert len(got) == 3
    for (pa, _, ca, qa), (k, ce, qe) in zip(got, expect):
        assert pa == k
        np.testing.assert_array_equal(ca, ce)
        np.testing.assert_array_equal(qa, qe)


def test_stray_npy_in_checkpoint_dir(tmp_path):
    """a plain .npy file beside the manifests is not a manifest (np.load returns an ndarray) and does
    not break _remove_unlisted."""
    from covid_spings_variant_caller_amd import live_variant_caller as LV
    stray = tmp_path / "stray.npy"
    np.save(str(stray), np.arange(5))
    assert _read_manifest(str(stray)) is None
    (tmp_path / "spgck-z-0-1.spgck").write_bytes(b"x")
    LV._remove_unlisted(str(tmp_path), {"spgck-z-0-1.spgck"})
    assert not (tmp_path / "spgck-z-0-1.spgck").exists() and stray.exists()
