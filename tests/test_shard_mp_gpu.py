"""Multi-GPU path with the HIP engine: 2 fresh processes (torch.distributed gloo, both ranks on
device 0 of the one-GPU test box) each run a coordinate-sharded ShardedEngine (shard.py) over every
batch, then the single gather of the call tables (shard.gather_candidates); rank 0's merged table must
equal a single engine's call table (SURVEY §8 e).  The RCCL branch is the same call with
backend "nccl" and device tensors (bench.py --gpus N)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import spings  # noqa: F401

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _batches():
    from covid_spings_variant_caller_amd import synth
    L = 6000
    ref = synth.reference(L, seed=61)
    bs = [synth.pileup(L, 400, seed=62, ref=ref, snv_every=41, lo=0, hi=4000),          # deep
          synth.pileup(L, 60, seed=63, ref=ref, snv_every=41, lo=1500, hi=L),            # shallow run
          synth.pileup(L, 80, seed=64, ref=ref, snv_every=37, lo=0, hi=L, max_depth=70)]
    return ref, bs


def _worker(rank, world, port, q):
    import torch.distributed as dist
    from covid_spings_variant_caller_amd import shard
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ref, batches = _batches()
    lo, hi = shard.partition(batches[0][1], world, batches[0][0], span=(0, len(ref)))[rank]
    eng = shard.ShardedEngine(lo, hi, ref, device=0)
    for b in batches:
        eng.accumulate(*b)
    merged = eng.gather()
    if rank == 0:
        q.put(merged.tobytes())
    eng.engine.close()
    dist.destroy_process_group()


def test_two_process_sharded_hip_engines_gather_matches_single_engine():
    from covid_spings_variant_caller_amd import _native as N
    from covid_spings_variant_caller_amd.engine import PileupEngine
    ref, batches = _batches()
    single = PileupEngine(len(ref), 30, 10, 5, 0.10, device=0, reference=ref, calls_only=True)
    for b in batches:
        single.accumulate(*b)
    single.finalize()
    want = single.candidates()
    single.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = np.frombuffer(q.get(timeout=180), dtype=N.CANDIDATE_DTYPE)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert len(want) > 20
    for k in ("pos", "dp", "ad", "pl", "score", "ref", "alt", "first_batch", "rank", "gl_zero"):
        np.testing.assert_array_equal(got[k], want[k], err_msg=k)
    np.testing.assert_allclose(got["gl"], want["gl"], rtol=1e-9, atol=0)
    np.testing.assert_allclose(got["qual"], want["qual"], rtol=1e-9, atol=0)
