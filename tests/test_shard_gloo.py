"""Multi-GPU path on CPU (gloo, world size 2): coordinate partition, per-rank batch slices, the
single gather of the call tables and the rank-0 merge reproduce the single-process call table.
Each rank's engine is stood in for by the C oracle (this container has no GPU); the GPU engine
itself is covered by the -m gpu tests."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import spings  # noqa: F401
from covid_spings_variant_caller_amd import _native as N
from covid_spings_variant_caller_amd import shard, synth


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _batches(ref):
    a = synth.pileup(len(ref), 60, seed=3, ref=ref, snv_every=37, lo=0, hi=700, read_len=50)
    b = synth.pileup(len(ref), 45, seed=4, ref=ref, snv_every=37, lo=300, hi=1000, read_len=50)
    return [a, b]


def _oracle_records(ref, batches, lo, hi, seq_of):
    """C-oracle stand-in for a rank's engine over [lo, hi): CANDIDATE_DTYPE records."""
    from oracle.c_oracle import COracle
    o = COracle(ref, 30, 10, 5, 0.10)
    first = {}
    for g, (pb, off, c, q) in enumerate(batches, start=1):
        spb, soff, sc, sq = shard.slice_batch(pb, off, c, q, lo, hi)
        if len(soff) > 1 and int(soff[-1]) > 0:
            o.accumulate(spb, soff, sc, sq)
            for k in range(len(soff) - 1):
                if soff[k + 1] > soff[k]:
                    first.setdefault(spb + k, seq_of(g))
    o.finalize()
    v = o.variants_array()
    out = np.zeros(len(v), N.CANDIDATE_DTYPE)
    for name in ("dp", "ad", "pl", "score", "ref", "alt", "gl_zero", "gl", "gl_linear", "qual"):
        out[name] = v[name]
    out["pos"] = v["start"]
    out["first_batch"] = [first[int(p)] for p in v["start"]]
    out["rank"] = [sum(1 for j in range(i) if v["start"][j] == v["start"][i]) for i in range(len(v))]
    return out


def _worker(rank, world, port, ref, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    batches = _batches(ref)
    # cut on the entries of the first batch, as a job would on its first sample
    lo, hi = shard.partition(batches[0][1], world, batches[0][0], span=(0, len(ref)))[rank]
    recs = _oracle_records(ref, batches, lo, hi, lambda g: g)
    merged = shard.gather_candidates(recs)
    if rank == 0:
        q.put(merged.tobytes())
    dist.destroy_process_group()


def test_partition_balances_entries():
    off = np.concatenate([[0], np.cumsum(np.r_[np.full(100, 10), np.full(100, 1000), np.full(100, 10)])])
    parts = shard.partition(off, 4, pos_begin=5)
    assert parts[0][0] == 5 and parts[-1][1] == 305
    assert all(parts[i][1] == parts[i + 1][0] for i in range(3))
    ent = [int(off[h - 5] - off[l - 5]) for l, h in parts]
    assert max(ent) - min(ent) <= 1000 + 10


def test_slice_batch_roundtrip():
    ref = synth.reference(500, seed=2)
    pb, off, c, q = synth.pileup(500, 30, seed=1, ref=ref, lo=20, hi=480, read_len=40)
    pieces = [shard.slice_batch(pb, off, c, q, lo, hi) for lo, hi in shard.partition(off, 3, pb)]
    assert np.array_equal(np.concatenate([p[2] for p in pieces]), c)
    assert np.array_equal(np.concatenate([p[3] for p in pieces]), q)
    assert sum(len(p[1]) - 1 for p in pieces) == len(off) - 1


def test_gloo_world2_gather_matches_single_process():
    from oracle.c_oracle import build
    build()
    ref = synth.reference(1000, seed=9)
    batches = _batches(ref)
    single = _oracle_records(ref, batches, 0, len(ref), lambda g: g)
    single = shard.merge_candidates([single])
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, ref, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = np.frombuffer(q.get(timeout=120), dtype=N.CANDIDATE_DTYPE)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert len(single) > 5
    for k in ("pos", "dp", "ad", "pl", "score", "ref", "alt", "first_batch", "rank"):
        np.testing.assert_array_equal(got[k], single[k], err_msg=k)
    np.testing.assert_array_equal(got["gl"], single["gl"])
    np.testing.assert_array_equal(got["qual"], single["qual"])
