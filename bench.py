"""Benchmark: pileup positions/s at 10,000x depth on 1..8 MI355X (BASELINE.json metric).

One step = one pass of the hot path over one batch: reset the accumulators (new sample), accumulate
the batch's CSR pileup (HBM-resident, borrowed), finalize (call table), and — for N > 1 — gather the
call tables to rank 0 (RCCL over xGMI).  Headline workload (BASELINE metric point): synthetic
SARS-CoV-2 (L = 29,903), 10,000x depth, 150-bp reads, uncapped.  Weak scaling: with N GPUs a step
processes N samples; rank r owns the r-th coordinate range of every sample.

Also on the same line (nested, never `value`), one per BASELINE config:
* ``parity_mode``: the metric point with pysam's max_depth 8,000 (E = 2.36e8);
* ``sars1k`` (config 2): SARS-CoV-2 at 1,000x, 64 samples stacked per GPU step (one sample is ~10 us of
  HBM traffic: SURVEY §8 d batches >= 64 samples per measurement);
* ``sars100k`` (config 3): 100,000x uncapped (the deep-column stress) and, nested, at max_depth 8,000;
* ``config4`` (config 4): 10,000 BAM-sized 100x samples as the per-BAM batches the drop-in produces, accumulated
  into one memory and finalized per step (the headline ``value``), the per-BAM finalize loop of
  vc_queue.py:142-144 (``per_bam_finalize``), and the column-major layout as an aside; coordinate-sharded over
  the N ranks (each rank: its range of every BAM);
* ``chr1_30x`` (config 5);
* ``multi_device``: the drop-in's own multi-GPU path (spg_multi, one process over devices 0..N-1: the same N stacked
  samples cut at equal entries, one ncclGather per step) — run by rank 0 while the other ranks wait (always at N > 1);
* ``end_to_end`` (host BAM -> calls) and ``cpu_baseline`` (the oracle restatements on host cores).

Output: rank 0 prints ONE compact JSON line (compact_line: the headline keys, roofline, a compact cpu_baseline and
{value, ms_per_step, frac} per nested leg, under LINE_LIMIT bytes); the full nested result goes to --detail-out.

``--gpus N`` without a launcher (no WORLD_SIZE in the environment) starts N rank processes of this script before
anything touches a GPU (127.0.0.1 rendezvous), as ``torch.distributed.run --nproc-per-node N`` would.

Timing: W untimed warm-up steps; then --reps measurements, each of exactly K = --steps steps between barrier + device
synchronize, max over ranks; the median measurement is reported (the nested legs: measurements of >= --leg-min-ms).  The dominant kernel's duration comes from HIP events on the engine's stream (every
--time-every-th step, so the events do not idle the GPU between steps).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_HBM = 8.0e12          # B/s per MI355X (MI355X_MICROARCH.md: 8.0 TB/s spec)
L_SARS = 29903


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20, help="minimum steps per timed measurement")
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--reps", type=int, default=20, help="timed measurements (median reported)")
    ap.add_argument("--min-ms", type=float, default=0.0,
                    help="headline: minimum duration of one measurement (0 = each measurement is exactly --steps steps)")
    ap.add_argument("--leg-min-ms", type=float, default=100.0, help="nested legs: minimum duration of one measurement")
    ap.add_argument("--workload", default="sars10k", choices=["sars10k", "sars1k", "sars100k", "chr1_30x", "sars_many"],
                    help="sars_many: BASELINE config 4 as the main line (the --many-* options)")
    ap.add_argument("--depth", type=float, default=0.0, help="override the workload's depth")
    ap.add_argument("--length", type=int, default=0, help="override the workload's reference length")
    ap.add_argument("--max-depth", type=int, default=0, help="0 = uncapped; 8000 = pysam parity cap")
    ap.add_argument("--no-parity", action="store_true", help="skip the max_depth 8000 nested line")
    ap.add_argument("--many-batches", type=int, default=10000, help="config 4 samples (0 = skip)")
    ap.add_argument("--many-depth", type=float, default=100.0)
    ap.add_argument("--runs-batches", type=int, default=10000,
                    help="config 4 as per-BAM CSR batches (the product path, counted mode; the headline); 0 = skip")
    ap.add_argument("--per-bam-bams", type=int, default=10000,
                    help="config 4's per-BAM finalize loop (vc_queue.py:142-144) over the first N BAMs; 0 = skip")
    ap.add_argument("--no-chr1", action="store_true", help="skip the nested chr1 30x line (BASELINE config 5)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-positions", type=int, default=6000)
    ap.add_argument("--no-e2e", action="store_true", help="skip the end-to-end BAM -> calls leg")
    ap.add_argument("--time-every", type=int, default=8,
                    help="HIP events around the accumulate kernel on every K-th timed step")
    ap.add_argument("--e2e-threads", type=int, default=0,
                    help="host threads of the end-to-end plan (0 = the per-GPU share of an 8-GPU node, "
                         "len(sched_getaffinity) // 8, capped by the process's cgroup CPU quota)")
    ap.add_argument("--e2e-bams", type=int, default=4, help="BAMs per end-to-end stream")
    ap.add_argument("--e2e-many", type=int, default=64,
                    help="config 4 end to end: 100x SARS-CoV-2 BAM files through process_bams (0 = skip)")
    ap.add_argument("--full-table", action="store_true", help="also accumulate every table GL term")
    ap.add_argument("--legs", default="parity,sars1k,sars100k,sars100k_capped,config4,chr1,multi,e2e,cpu",
                    help="nested legs of the default sars10k line (comma list; 'none' = the main point only)")
    ap.add_argument("--no-main", action="store_true", help="profiling: skip the main point (nested legs only)")
    ap.add_argument("--sars1k-samples", type=int, default=64, help="stacked samples per GPU step at 1,000x")
    ap.add_argument("--multi-helper", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--multi-timeout", type=float, default=300.0, help="time limit of the multi-device leg at N > 1 (s)")
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend for N > 1 (nccl = RCCL; "
                                                      "gloo only to exercise the path on one GPU)")
    ap.add_argument("--detail-out", default=os.path.join("gpurun_out", "bench_detail_n{n}.json"),
                    help="file for the full nested result (the printed line is the compact form); '' = none")
    return ap.parse_args()


WORKLOADS = {   # BASELINE.json configs (the metric is quoted on sars10k)
    "sars10k": (L_SARS, 10000.0, "NC_045512.2"),
    "sars1k": (L_SARS, 1000.0, "NC_045512.2"),
    "sars100k": (L_SARS, 100000.0, "NC_045512.2"),
    "chr1_30x": (248956422, 30.0, "chr1"),
}


def rank_envs(n: int, port: int, base=None):
    """The environments of n local ranks (what torch.distributed.run exports), rendezvous on 127.0.0.1:port."""
    base = dict(os.environ if base is None else base)
    return [dict(base, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                 MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port)) for r in range(n)]


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return int(s.getsockname()[1])


def spawn_ranks(n: int, argv) -> int:
    """`bench.py --gpus N` started without a launcher (no WORLD_SIZE): start N rank processes of this script — one per
    GPU, before this process has touched any GPU — and return the first failing exit code (0 when all succeed).
    Rank 0 prints the JSON line on the inherited stdout.  If one rank fails, the others are terminated (by PID)."""
    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env)
             for env in rank_envs(n, free_port())]
    rc = 0
    try:
        pending = list(procs)
        while pending:
            for p in list(pending):
                r = p.poll()
                if r is None:
                    continue
                pending.remove(p)
                if r != 0 and rc == 0:
                    rc = r
                    for q in pending:
                        q.terminate()
            if pending:
                time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    return rc


class _StdoutToStderr:
    """fd 1 pointed at stderr for the duration (gloo prints its "connected to N peer ranks" lines on stdout: rank 0's
    stdout must hold exactly the one JSON line)."""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)

    def __exit__(self, *a):
        sys.stdout.flush()
        os.dup2(self.saved, 1)
        os.close(self.saved)


class Dist:
    """torch.distributed helpers (no-ops at N = 1).  Beside the data path's group (RCCL for nccl), a gloo group for
    host-side waits: ranks that sit out a leg rank 0 runs on every device (spg_multi) wait there, not in an RCCL
    collective that would hold a kernel on their GPU."""

    def __init__(self, world, rank, backend, device):
        self.world, self.rank, self.backend, self.device = world, rank, backend, device
        self.dist = None
        self.cpu_group = None
        if world > 1:
            import torch
            import torch.distributed as dist
            with _StdoutToStderr():
                if backend == "nccl":
                    dist.init_process_group("nccl", device_id=device)
                    self.cpu_group = dist.new_group(backend="gloo")
                else:
                    dist.init_process_group(backend)
            self.dist = dist
            self.tdev = device if backend == "nccl" else torch.device("cpu")

    def barrier(self):
        if self.dist is not None:
            self.dist.barrier()

    def host_barrier(self):
        if self.dist is not None:
            self.dist.barrier(group=self.cpu_group)

    def all_gather_object(self, obj):
        if self.dist is None:
            return [obj]
        out = [None] * self.world
        self.dist.all_gather_object(out, obj, group=self.cpu_group)
        return out

    def max(self, x: float) -> float:
        if self.dist is None:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64, device=self.tdev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def close(self):
        if self.dist is not None:
            self.dist.destroy_process_group()


def measure(D, step, eng, K_min, reps, min_ms, every):
    """reps measurements of K steps each (K >= K_min, >= min_ms of steps); max over ranks.  Returns
    (K, per-measurement seconds, accumulate-kernel ms samples)."""
    import torch
    eng.sync()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    flush = getattr(step, "flush", lambda: None)     # outstanding asynchronous gathers
    for k in range(3):
        step(k)
    flush()
    eng.sync()
    est = D.max((time.perf_counter() - t0) / 3)
    K = max(K_min, int(math.ceil(min_ms * 1e-3 / max(est, 1e-7))))
    # re-estimate K from timed batches of K steps (the 3 steps above carry first-call overheads), so that
    # every measurement lasts >= min_ms
    for _ in range(3):
        torch.cuda.synchronize()
        D.barrier()
        t0 = time.perf_counter()
        for k in range(K):
            step(k)
        flush()
        eng.sync()
        torch.cuda.synchronize()
        t = D.max(time.perf_counter() - t0)
        # (a timed measurement runs a few % faster than this calibration batch: 15 % margin)
        if t >= 1.15 * min_ms * 1e-3:
            break
        K = max(K + 1, int(math.ceil(K * min_ms * 1.25e-3 / max(t, 1e-9))))
    eng.kernel_times(4096)
    times, acc, enq = [], [], []
    for _ in range(reps):
        eng.set_timing(0)
        torch.cuda.synchronize()
        D.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(K):
            eng.set_timing(1 if k % every == 0 else 0)
            step(k)
        enq.append(time.perf_counter() - t0)       # host time to enqueue the K steps
        flush()                                    # the last steps' gathers complete inside the window
        torch.cuda.synchronize()                   # (every stream of the device, the engine's included)
        D.barrier()
        times.append(D.max(time.perf_counter() - t0))
        a, _ = eng.kernel_times(4096)
        acc.extend(a[a > 0].tolist())
    measure.host_enqueue_ms_per_step = float(np.median(enq)) / K * 1e3
    return K, np.array(times), np.array(acc)


def finalize_ms(step, eng, n=8):
    eng.set_timing(2)
    for k in range(n):
        step(k)
    getattr(step, "flush", lambda: None)()
    eng.sync()
    _, f = eng.kernel_times(4096)
    eng.set_timing(0)
    return float(np.mean(f[f > 0])) if (f > 0).any() else 0.0


def build_shard(rank, world, L, depth, max_depth, device, samples=1, distinct=None):
    """This rank's coordinate range of each of `world` x `samples` samples, generated natively
    (libspings_pileup spp_synth_batch: SURVEY §8 d read model) and concatenated in HBM.  The samples are
    STACKED: sample s owns positions [s C, (s + 1) C) of the engine's coordinate space, so one context holds
    `samples` independent memories and one launch processes them all (SURVEY §8 d: batches of >= 64 samples
    for the 1,000x config, whose single sample is ~10 us of HBM traffic).  Only `distinct` samples are
    generated (seeds 2, 3, ...); the others repeat them (the kernel reads every copy)."""
    import torch
    from covid_spings_variant_caller_amd import synth
    from covid_spings_variant_caller_amd.pileup import synth_batch
    ref = synth.reference(L, seed=1)
    shard = (L + world - 1) // world
    lo, hi = rank * shard, min(L, (rank + 1) * shard)
    n = world * samples
    distinct = n if distinct is None else max(1, min(n, distinct))
    threads = min(16, len(os.sched_getaffinity(0)))
    gen = []
    for s in range(distinct):
        b = synth_batch(ref, depth, lo=lo, hi=hi, seed=2 + s, n_threads=threads, max_depth=max_depth)
        gen.append((b.offsets.copy(), torch.from_numpy(b.codes).to(device), torch.from_numpy(b.quals).to(device)))
        b.close()
    offs, dc, dq = [np.zeros(1, np.uint64)], [], []
    base = 0
    for s in range(n):
        o, c, q = gen[s % distinct]
        offs.append(o[1:] + np.uint64(base))
        base += int(o[-1])
        dc.append(c)
        dq.append(q)
    pad = torch.zeros(16, dtype=torch.uint8, device=device)
    d_c = torch.cat(dc + [pad + 0xFF])
    d_q = torch.cat(dq + [pad])
    del gen, dc, dq
    off = np.concatenate(offs)
    d_off = torch.from_numpy(off.view(np.int64).copy()).to(device)
    return ref, ref[lo:hi] * n, off, d_off, d_c, d_q, int(base)


def kernel_name(E, C, calls_only=True):
    """The accumulate kernel the engine picks for one batch of E entries over C columns
    (csrc/spg_api.cpp add_batch / flush_run) and its PMC summary key."""
    if E <= 40 * C and calls_only:   # one shallow batch into a fresh memory, fused with the calls-only finalize
        return "k_acc_lite (+ k_acc_seg<1> for columns >= 128 entries)", "spg::k_acc_lite"
    if E < 256 * C:
        return "k_acc_tile (+ k_acc_seg<1> for columns >= 128 entries)", "spg::k_acc_tile"
    if E < 4096 * C and calls_only:   # a lone mid-depth batch (1,000x): counted, the listed columns folded exactly
        lpc = 4
        while lpc < 64 and E / C / 16.0 / lpc > 2.5:
            lpc *= 2
        return (f"k_count_cols<{lpc},4> + k_acc_seg<1> over the listed columns (+ sparse k_finalize)",
                f"spg::k_count_cols<{lpc}, 4>")
    nt = 2 * E > (192 << 20)
    return (f"k_acc_seg<4,true,4,{'true' if nt else 'false'}> (spg_accumulate{'; non-temporal loads' if nt else ''})",
            "spg::k_acc_seg<4, true")


TRAFFIC_NOTE = ("not read in this run: HBM bytes per launch looked up from the newest committed PMC summary of this "
                "kernel on this workload (profiles/rNN_*_pmc.json: rocprofv3 --pmc FETCH_SIZE x2 + WRITE_SIZE, "
                "tools/summarize_prof.py); null when none was committed")


def pmc_traffic(key, E, with_source=False):
    """HBM bytes per launch of the accumulate kernel from the newest committed PMC summary
    (profiles/rNN_*pmc.json, tools/summarize_prof.py over rocprofv3 --pmc passes of this bench:
    FETCH_SIZE x2 + WRITE_SIZE), when it was measured on this workload; else None.  A lookup, not a counter read in
    this run (the line labels it: traffic_source)."""
    import glob
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc.json")), reverse=True):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        for k, v in d.items():
            if k.startswith(key) and v.get("entries") == E:
                val = v.get("hbm_bytes_per_launch")
                return (val, os.path.relpath(f, ROOT)) if with_source else val
    return (None, None) if with_source else None


def pmc_traffic_sum(keys, E):
    """Sum of pmc_traffic over the kernels of one step (each from the newest summary measured on this
    workload); None when any of them was not measured."""
    vals = [pmc_traffic(k, E) for k in keys]
    return None if any(v is None for v in vals) else float(sum(vals))


def run_point(args, D, L, depth, max_depth, local, world, rank, contig, samples=1, distinct=None, min_ms=None):
    """The metric point (`samples` stacked samples per GPU per step, each coordinate-sharded): returns the
    result dict."""
    import torch
    from covid_spings_variant_caller_amd.engine import PileupEngine
    dev = torch.device("cuda", local)
    t_gen = time.perf_counter()
    ref, vref, off, d_off, d_c, d_q, E = build_shard(rank, world, L, depth, max_depth, dev, samples, distinct)
    C = len(off) - 1
    t_gen = time.perf_counter() - t_gen
    # calls-only engine (SPG_P_CALLS_ONLY): the call table prepare_variants() returns, exactly
    eng = PileupEngine(C, 30, 10, 5, 0.10, device=local, reference=vref, calls_only=not args.full_table)
    eng.reset()
    eng.accumulate(0, d_off, d_c, d_q, borrow=True, n_entries=E)
    eng.finalize()
    n_cand, n_replay = eng.counts()
    # call-table gather: persistent double buffers, sized from this first pass (KBs per step).  The
    # gather of step k runs asynchronously (RCCL's stream) while step k + 1 computes; a buffer is
    # reused two steps later, after its gather has completed.
    cap = max(64, 4 * n_cand)
    cap = int(D.max(cap))
    rec = 56
    gdev = dev if args.backend == "nccl" else torch.device("cpu")
    gbufs = [torch.zeros(cap * rec + 8, dtype=torch.uint8, device=dev) for _ in range(2)]
    sends = gbufs if args.backend == "nccl" else [torch.zeros_like(b, device="cpu") for b in gbufs]
    recvs = [[torch.zeros_like(sd) for _ in range(world)] if (world > 1 and rank == 0) else None for sd in sends]
    pending = [None, None]

    def step(k):
        eng.reset()
        eng.accumulate(0, d_off, d_c, d_q, borrow=True, n_entries=E)
        eng.finalize()
        if world > 1:
            j = k & 1
            if pending[j] is not None:
                pending[j].wait()                       # nccl: torch's stream waits on the gather
                pending[j] = None
                # the engine's stream (which writes the buffer) waits on torch's stream
                eng._torch_stream().wait_stream(torch.cuda.current_stream(dev))
            eng.copy_candidates_device(gbufs[j], cap=cap)
            if args.backend != "nccl":
                sends[j].copy_(gbufs[j])                # device -> persistent host buffer (gloo)
            pending[j] = D.dist.gather(sends[j], recvs[j], dst=0, async_op=True)   # RCCL over xGMI

    def flush():
        waited = False
        for j in range(2):
            if pending[j] is not None:
                pending[j].wait()
                pending[j] = None
                waited = True
        if waited:
            torch.cuda.synchronize(dev)

    step.flush = flush

    for k in range(args.warmup):
        step(k)
    K, times, acc = measure(D, step, eng, args.steps, args.reps, args.min_ms if min_ms is None else min_ms,
                            max(1, args.time_every))
    fin = finalize_ms(step, eng)
    gathered = None
    if world > 1:
        # the gathered table must equal every rank's own table (count and bytes)
        step(0)
        flush()
        eng.sync()
        torch.cuda.synchronize()
        send, gather_buf, recv = sends[0], gbufs[0], recvs[0]
        mine = np.frombuffer(send.cpu().numpy().tobytes(), np.uint8) if args.backend != "nccl" else \
            gather_buf.cpu().numpy()
        n_mine = int(mine[:8].view(np.uint64)[0])
        allmine = [torch.from_numpy(mine[:8 + n_mine * rec].copy()).to(gdev)]
        sizes = torch.tensor([8 + n_mine * rec], dtype=torch.int64, device=gdev)
        all_sizes = [torch.zeros_like(sizes) for _ in range(world)]
        D.dist.all_gather(all_sizes, sizes)
        if rank == 0:
            gathered = 0
            for r in range(world):
                got = recv[r].cpu().numpy()
                n = int(got[:8].view(np.uint64)[0])
                assert 8 + n * rec == int(all_sizes[r].item()), "gathered count differs from the rank's table"
                gathered += n
            assert np.array_equal(recv[0].cpu().numpy()[:8 + n_mine * rec], mine[:8 + n_mine * rec]), \
                "gathered bytes differ from rank 0's table"
        # every rank sends its table bytes to rank 0 for a byte comparison
        buf = torch.zeros(8 + cap * rec, dtype=torch.uint8, device=gdev)
        buf[:8 + n_mine * rec] = allmine[0]
        outs = [torch.zeros_like(buf) for _ in range(world)] if rank == 0 else None
        D.dist.gather(buf, outs, dst=0)
        if rank == 0:
            for r in range(world):
                a, b = outs[r].cpu().numpy(), recv[r].cpu().numpy()
                n = int(a[:8].view(np.uint64)[0])
                assert np.array_equal(a[:8 + n * rec], b[:8 + n * rec]), f"rank {r}: gathered bytes differ"
    med = float(np.median(times))
    t_acc = float(np.mean(acc)) * 1e-3 if len(acc) else float("nan")
    # bytes the accumulate + finalize must move: base_code + qual + u64 offsets + REF chars read, the
    # calls-only candidate records (56 B) written
    algo_bytes = 2 * E + 8 * (C + 1) + C + 56 * n_cand
    eng.close()
    del d_off, d_c, d_q
    torch.cuda.empty_cache()
    return {
        "value": world * samples * L * K / med, "ms_per_step": med / K * 1e3, "steps": K, "reps": len(times),
        "E": E, "C": C,
        "measurements_ms": [round(t * 1e3, 3) for t in times], "t_gen": t_gen,
        "kernel_ms": t_acc * 1e3, "kernel_ms_median": float(np.median(acc)) if len(acc) else None,
        "kernel_samples": int(len(acc)), "algo_bytes": algo_bytes, "achieved": algo_bytes / t_acc,
        "finalize_ms": fin, "n_cand": n_cand, "n_replay": n_replay, "gathered": gathered,
        "host_enqueue_ms_per_step": measure.host_enqueue_ms_per_step,
    }


def multi_devices(world: int, backend: str):
    """The devices rank 0's spg_multi leg spans: one per rank (0..N-1); with a non-RCCL backend on fewer GPUs (a
    functional run of the N > 1 path) the ranks' devices modulo the GPUs present, as the ranks themselves map them."""
    import torch
    n_dev = max(1, torch.cuda.device_count())
    return [d if backend == "nccl" else d % n_dev for d in range(world)]


def run_multi_device(args, world, L, depth, max_depth):
    """The drop-in's own multi-GPU path (LiveVariantCaller(devices=...) -> multi.MultiEngine -> spg_multi_*), driven
    by ONE process over devices 0..N-1: the same weak-scaling step as the main point — N samples stacked into one
    coordinate space of N x L positions, cut at equal entries (spg_multi_plan), each device holding its slice in its
    own HBM — with reset + spg_multi_accumulate_slices (borrowed) + spg_multi_finalize + spg_multi_get_candidates (the
    merged call table: one ncclGather over xGMI to devices[0] when the devices are distinct, device copies when one GPU
    stands in for several) per step.  Unlike the per-rank path, every step ends with the table on the host (what
    prepare_variants returns), so the host's launch and gather latency are inside the step."""
    import torch
    from covid_spings_variant_caller_amd import synth
    from covid_spings_variant_caller_amd.multi import MultiEngine
    from covid_spings_variant_caller_amd.pileup import synth_batch
    devices = multi_devices(world, args.backend)
    ref = synth.reference(L, seed=1)
    t0 = time.perf_counter()
    distinct = min(world, 2)
    threads = min(16, len(os.sched_getaffinity(0)))
    gen = []
    for s in range(distinct):
        b = synth_batch(ref, depth, lo=0, hi=L, seed=2 + s, n_threads=threads, max_depth=max_depth)
        gen.append((b.offsets.astype(np.uint64).copy(), b.codes.copy(), b.quals.copy()))
        b.close()
    samples = [gen[s % distinct] for s in range(world)]
    full_off = np.zeros(world * L + 1, np.uint64)
    base = 0
    for s, (o, _, _) in enumerate(samples):
        full_off[s * L + 1:(s + 1) * L + 1] = o[1:] + np.uint64(base)
        base += int(o[-1])
    E = base
    mm = MultiEngine(devices, world * L, 30, 10, 5, 0.10, reference=ref * world, calls_only=True)
    cuts = mm.plan(0, full_off)
    slices, hold = [], []
    for d, dev in enumerate(devices):
        lo, hi = int(cuts[d]), int(cuts[d + 1])
        pc, pq, lens = [], [], []
        for s in range(world):
            a, b = max(lo, s * L), min(hi, (s + 1) * L)
            if b <= a:
                continue
            o, c, q = samples[s]
            pc.append(c[int(o[a - s * L]):int(o[b - s * L])])
            pq.append(q[int(o[a - s * L]):int(o[b - s * L])])
            lens.append(np.diff(o[a - s * L:b - s * L + 1].astype(np.int64)))
        tdev = torch.device("cuda", dev)
        off_d = np.zeros(hi - lo + 1, np.uint64)
        np.cumsum(np.concatenate(lens), out=off_d[1:])
        pad = np.zeros(16, np.uint8)
        t_off = torch.from_numpy(off_d.view(np.int64)).to(tdev)
        t_c = torch.from_numpy(np.concatenate(pc + [pad + 0xFF])).to(tdev)
        t_q = torch.from_numpy(np.concatenate(pq + [pad])).to(tdev)
        slices.append((lo, t_off, t_c, t_q))
        hold.append((t_off, t_c, t_q))
    del gen, samples
    for dev in set(devices):
        torch.cuda.synchronize(dev)
    t_gen = time.perf_counter() - t0

    pend = []
    got = []
    desc = mm.prepare_slices(0, full_off, slices)

    def step():
        # step k's table is enqueued (spg_multi_get_candidates_async: device copies, the gather, one copy into pinned
        # host memory) and step k - 1's is waited for and merged: step k's launches are out before then
        mm.reset()
        mm.accumulate_slices(0, full_off, desc, borrow=True)
        mm.finalize()
        pend.append(mm.candidates_async())
        if len(pend) > 1:
            got.append(mm.wait_candidates(pend.pop(0)))

    def flush():
        while pend:
            got.append(mm.wait_candidates(pend.pop(0)))

    mm.reset()
    mm.accumulate_slices(0, full_off, slices, borrow=True)
    mm.finalize()
    calls = mm.candidates()                      # (synchronous: sizes the table copies)
    assert np.array_equal(mm.partition(), cuts), "spg_multi re-planned the stacked sample's cuts"
    for _ in range(max(1, args.warmup)):
        step()
    flush()
    assert all(np.array_equal(g, calls) for g in got), "the pipelined tables differ from the synchronous one"
    got.clear()
    mm.sync()
    t = time.perf_counter()
    for _ in range(3):
        step()
    flush()
    est = (time.perf_counter() - t) / 3
    K = max(args.steps, int(math.ceil(args.leg_min_ms * 1e-3 / max(est, 1e-7))))
    mm.kernel_times()
    mm.set_timing(1)
    times, kern = [], []
    for _ in range(max(5, args.reps // 2)):
        mm.sync()
        got.clear()
        t = time.perf_counter()
        for _ in range(K):
            step()
        flush()                                  # every step's table is on the host inside the window
        mm.sync()
        times.append(time.perf_counter() - t)
        assert len(got) == K and np.array_equal(got[-1], calls), "pipelined table"
        per_dev = [a for a, _ in mm.kernel_times()]
        n = min(len(a) for a in per_dev)
        if n:
            kern.extend(np.max(np.stack([a[-n:] for a in per_dev]), axis=0).tolist())   # slowest device per step
    mm.set_timing(0)
    med = float(np.median(times))
    t_k = float(np.mean(kern)) * 1e-3 if kern else float("nan")
    algo = 2 * E + 8 * (world * L + len(devices)) + world * L + 56 * len(calls)
    per_dev_bytes = algo / len(devices)
    mm.close()
    del slices, hold
    torch.cuda.empty_cache()
    return {"workload": f"{world} samples x {L} positions at {depth:.0f}x ({'uncapped' if not max_depth else f'max_depth {max_depth}'}) "
                        f"stacked into one spg_multi coordinate space, sliced at equal-entry cuts, slices resident in "
                        f"each device's HBM (borrowed)",
            "devices": devices, "rccl": len(set(devices)) == len(devices) and len(devices) > 1,
            "cuts": [int(x) for x in cuts], "value": world * L * K / med, "unit": "positions/s",
            "ms_per_step": med / K * 1e3, "steps": K * len(times), "steps_per_measurement": K,
            "measurement_ms": [round(x * 1e3, 3) for x in times], "entries_per_step": E, "datagen_s": t_gen,
            "calls_per_step": len(calls),
            "step": "spg_multi_reset + spg_multi_accumulate_slices + spg_multi_finalize + spg_multi_get_candidates_async "
                    "(the call table merged on the host by spg_multi_wait_candidates one step later; every step's table "
                    "is on the host inside the timed window)",
            "kernel_ms_slowest_device": t_k * 1e3,
            "roofline": {"bound": "hbm", "achieved": per_dev_bytes / t_k / 1e9, "peak": PEAK_HBM / 1e9, "unit": "GB/s",
                         "frac": per_dev_bytes / t_k / PEAK_HBM,
                         "frac_basis": "mean bytes per device / slowest device's accumulate kernel"}}


def multi_helper(args) -> int:
    """bench.py --multi-helper: wait for "go" on stdin (rank 0's signal, after the per-rank measurements), then run the
    multi-device leg over devices 0..WORLD_SIZE-1 and print its result as one JSON line."""
    go = sys.stdin.readline().strip()
    if go != "go":
        return 0
    world = int(os.environ.get("WORLD_SIZE", "1"))
    L, depth, _ = WORKLOADS[args.workload]
    L = args.length or L
    depth = args.depth or depth
    try:
        import spings  # noqa: F401
        out = run_multi_device(args, world, L, depth, args.max_depth)
    except Exception as e:
        out = {"error": f"{type(e).__name__}: {e}"}
    print(json.dumps(out), flush=True)
    return 0


def run_helper(helper, timeout_s: float):
    """Signal rank 0's helper and collect its JSON line; a helper past the time limit is killed (its PID) and the leg
    reported as timed out."""
    import threading
    out = {}

    def read():
        out["line"] = helper.stdout.readline()

    try:
        helper.stdin.write("go\n")
        helper.stdin.flush()
    except OSError as e:
        return {"error": f"helper: {e}"}
    th = threading.Thread(target=read, daemon=True)
    th.start()
    th.join(timeout_s)
    if th.is_alive():
        helper.kill()
        helper.wait()
        return {"error": f"multi-device leg did not finish within {timeout_s:.0f} s (helper killed)"}
    helper.wait(timeout=60)
    try:
        return json.loads(out.get("line") or "{}")
    except ValueError:
        return {"error": f"helper output: {out.get('line', '')[:200]!r}"}


def nested_point(args, D, workload, local, world, rank, max_depth=0, samples=1, distinct=None, step_frac=False):
    """Another BASELINE config as a nested line (never `value`): same step and timing as the main point.
    `step_frac`: the roofline fraction is taken over the whole step's kernels (accumulate + finalize launches),
    for paths where the finalize is a launch of its own (chr1: k_acc_lite + k_lite_fold + sparse k_finalize)."""
    L, depth, contig = WORKLOADS[workload]
    p = run_point(args, D, L, depth, max_depth, local, world, rank, contig, samples, distinct, min_ms=args.leg_min_ms)
    name, key = kernel_name(p["E"], p["C"], not args.full_table)
    frac_k = p["achieved"] / PEAK_HBM
    frac_s = p["algo_bytes"] / ((p["kernel_ms"] + p["finalize_ms"]) * 1e-3) / PEAK_HBM
    stack = (f"{samples} samples stacked per GPU per step (sample s = positions [s C, (s+1) C) of one context; "
             f"{distinct or samples * world} distinct, repeated)" if samples > 1 else "1 sample per GPU per step")
    return {"workload": f"{workload}: {contig} L={L}, {depth:.0f}x, 150-bp reads, "
                        f"{'uncapped' if not max_depth else f'max_depth {max_depth}'}, {stack} (coordinate-sharded x{world})",
            "value": p["value"], "unit": "positions/s", "ms_per_step": p["ms_per_step"], "steps": p["steps"] * p["reps"],
            "steps_per_measurement": p["steps"], "measurement_ms": p["measurements_ms"], "samples_per_gpu_step": samples,
            "entries_per_gpu_step": p["E"], "columns_per_gpu": p["C"],
            "datagen_s": p["t_gen"], "finalize_ms": p["finalize_ms"], "candidates_per_gpu_step": p["n_cand"],
            "replayed_positions_per_gpu_step": p["n_replay"],
            "roofline": {"bound": "hbm", "achieved": (frac_s if step_frac else frac_k) * PEAK_HBM / 1e9,
                         "peak": PEAK_HBM / 1e9, "unit": "GB/s", "frac": frac_s if step_frac else frac_k,
                         "frac_basis": "accumulate + finalize kernels" if step_frac else "accumulate kernel",
                         "algorithmic_bytes": p["algo_bytes"], "frac_kernel_only": frac_k, "frac_incl_finalize": frac_s,
                         "traffic": pmc_traffic(key, p["E"]), "kernel": name, "kernel_ms": p["kernel_ms"],
                         "kernel_ms_median": p["kernel_ms_median"], "kernel_samples": p["kernel_samples"]}}


def run_config4(args, D, local, world, rank):
    """BASELINE config 4: args.runs_batches BAM-sized samples (args.many_depth x, per-BAM cap 8,000) accumulated
    into one memory; this rank's coordinate range of every BAM.

    Headline (``value``): the product path — the per-BAM CSR batches one process_bam per BAM produces
    (live_variant_caller.py:54-72; LiveVariantCaller.process_bams), accumulated and finalized once per step
    (counted mode).  ``per_bam_finalize``: vc_queue.py:142-144's loop — process_bam then write_vcf's
    prepare_variants after EVERY BAM, the call table read back each time.  ``column_major_aside``: the same
    BAMs as one column-major multi-BAM batch (spg_accumulate_samples), a layout no product path produces
    (reported for comparison only)."""
    from covid_spings_variant_caller_amd import synth
    L = L_SARS
    ref = synth.reference(L, seed=1)
    shard = (L + world - 1) // world
    lo, hi = rank * shard, min(L, (rank + 1) * shard)
    res = run_config4_runs(args, D, local, world, rank, ref, lo, hi)
    if args.many_batches > 0:
        res["column_major_aside"] = run_config4_columns(args, D, local, world, rank, ref, lo, hi)
    return res


def run_config4_columns(args, D, local, world, rank, ref, lo, hi):
    """Config 4's BAMs as one column-major multi-sample batch (k_acc_seg over deep columns)."""
    import torch
    from covid_spings_variant_caller_amd.engine import PileupEngine
    from covid_spings_variant_caller_amd.synth_device import many_bams_columns
    dev = torch.device("cuda", local)
    L, C, B = L_SARS, hi - lo, args.many_batches
    t0 = time.perf_counter()
    d = many_bams_columns(ref, B, args.many_depth, seed=1000, lo=lo, hi=hi, max_depth=8000, device=dev)
    torch.cuda.synchronize()
    t_gen = time.perf_counter() - t0
    E = d.n_entries
    eng = PileupEngine(C, 30, 10, 5, 0.10, device=local, reference=ref[lo:hi], calls_only=True)

    def step(k):
        eng.reset()
        eng.accumulate_samples(0, d.offsets, d.first_sample, d.codes, d.quals, B, borrow=True, n_entries=E)
        eng.finalize()

    step(0)
    n_cand, n_replay = eng.counts()
    for k in range(args.warmup):
        step(k)
    K, times, acc = measure(D, step, eng, args.steps, args.reps, args.leg_min_ms, max(1, args.time_every))
    fin = finalize_ms(step, eng)
    med = float(np.median(times))
    t_acc = float(np.mean(acc)) * 1e-3 if len(acc) else float("nan")
    # bytes the kernel must move for this layout: base_code + qual + u64 offsets + u32 first-sample per column
    # read, 56-B candidate records written
    moved = 2 * E + 8 * (C + 1) + 4 * C + C + 56 * n_cand
    eng.close()
    del d
    torch.cuda.empty_cache()
    return {
        "workload": f"{B} synthetic SARS-CoV-2 BAMs x {args.many_depth:.0f}x as ONE column-major multi-BAM batch "
                    f"(spg_accumulate_samples; not a layout the drop-in produces), accumulated + finalized per step",
        "value": B * L * K / med, "unit": "positions/s (BAMs x L per step)",
        "ms_per_step": med / K * 1e3, "steps": K * len(times), "steps_per_measurement": K,
        "entries_per_gpu_step": E, "columns_per_gpu": C, "datagen_s": t_gen,
        "kernel": kernel_name(E, C)[0], "accumulate_ms": t_acc * 1e3, "accumulate_samples": int(len(acc)),
        "finalize_ms": fin, "candidates_per_gpu_step": n_cand, "replayed_positions_per_gpu_step": n_replay,
        "roofline": {"bound": "hbm", "achieved": moved / t_acc / 1e9, "peak": PEAK_HBM / 1e9, "unit": "GB/s",
                     "frac": moved / t_acc / PEAK_HBM, "algorithmic_bytes": moved,
                     "traffic": pmc_traffic(kernel_name(E, C)[1], E)}}


def run_config4_runs(args, D, local, world, rank, ref, lo, hi):
    """Config 4 as per-BAM CSR batches (batch-major, what one process_bam per BAM produces), counted at the
    finalize (counted mode: k_acc_lite_run + k_count_list + k_fold_hist + the sparse k_finalize); then the
    per-BAM finalize loop over the same batches."""
    import torch
    from covid_spings_variant_caller_amd.engine import PileupEngine
    from covid_spings_variant_caller_amd.synth_device import many_bams
    dev = torch.device("cuda", local)
    B, C, L = args.runs_batches, hi - lo, L_SARS
    t0 = time.perf_counter()
    data = many_bams(ref, B, args.many_depth, seed=1000, lo=lo, hi=hi, max_depth=8000, device=dev)
    torch.cuda.synchronize()
    t_gen = time.perf_counter() - t0
    recs = data.records(pos_begin=0)   # the engine covers this shard only
    E = int(data.n_entries.sum())
    eng = PileupEngine(C, 30, 10, 5, 0.10, device=local, reference=ref[lo:hi], calls_only=True)

    def step(k):
        eng.reset()
        eng.accumulate_records(recs)
        eng.finalize()

    step(0)
    n_cand = eng.counts()[0]
    final_calls = eng.candidates()
    K, times, acc = measure(D, step, eng, 1, max(5, args.reps // 4), args.leg_min_ms, 1)
    med = float(np.median(times))
    t_acc = float(np.mean(acc)) * 1e-3 if len(acc) else float("nan")
    # bytes the run must move: each BAM's base_code + qual + u64 offsets, the REF chars, the candidate records
    moved = 2 * E + 8 * B * (C + 1) + C + 56 * n_cand
    kname = "counted mode: k_acc_lite_run + k_count_list + k_fold_hist + sparse k_finalize"
    res = {"workload": f"{B} synthetic SARS-CoV-2 BAMs x {args.many_depth:.0f}x (per-BAM cap 8000, generated in HBM) "
                       f"as per-BAM CSR batches (what LiveVariantCaller.process_bams accumulates), accumulated into one "
                       f"memory + prepare_variants per step; coordinate-sharded x{world}",
           "bams": B, "value": B * L * K / med, "unit": "positions/s (BAMs x L per step)",
           "ms_per_step": med / K * 1e3, "steps": K * len(times), "steps_per_measurement": K,
           "measurement_ms": [round(t * 1e3, 3) for t in times],
           "entries_per_gpu_step": E, "columns_per_gpu": C, "datagen_s": t_gen, "kernel": kname,
           "accumulate_ms": t_acc * 1e3, "accumulate_samples": int(len(acc)), "candidates_per_gpu_step": n_cand,
           "roofline": {"bound": "hbm", "achieved": moved / t_acc / 1e9, "peak": PEAK_HBM / 1e9, "unit": "GB/s",
                        "frac": moved / t_acc / PEAK_HBM, "algorithmic_bytes": moved,
                        "traffic": pmc_traffic_sum(("spg::k_acc_lite_run", "spg::k_count_list", "spg::k_fold_hist",
                                                    "spg::k_finalize"), E)}}
    if args.per_bam_bams > 0:
        res["per_bam_finalize"] = per_bam_loop(args, D, eng, data, recs, min(B, args.per_bam_bams), C, final_calls)
    eng.close()
    del data
    torch.cuda.empty_cache()
    return res


def per_bam_loop(args, D, eng, data, recs, nb, C, final_calls):
    """vc_queue.py:142-144 without the file I/O: per BAM, accumulate its batch (process_bam's accumulate step), then
    prepare_variants (finalize + the call table read back to the host, as write_vcf needs it).  Every finalize
    after the first counts only the new BAM and re-folds only the positions that can call (incremental counted
    mode, from the first BAM on: no record-path run and no full-range finalize, `engine_paths` counts them)."""
    import torch
    eng.reset()
    eng.sync()
    eng.kernel_times(4096)
    eng.set_timing(2)
    lat, gpu = np.zeros(nb), np.zeros(nb)
    n_calls = np.zeros(nb, np.int64)
    pc0 = eng.path_counters()
    D.barrier()
    t0 = time.perf_counter()
    done = 0
    for i in range(nb):
        t = time.perf_counter()
        eng.accumulate_records(recs[i:i + 1])
        eng.finalize()
        calls = eng.candidates()                    # device -> host (synchronises the step)
        lat[i] = time.perf_counter() - t
        n_calls[i] = len(calls)
        if (i + 1) % 128 == 0 or i == nb - 1:       # the timing ring holds 256 finalizes
            a, f = eng.kernel_times(4096)
            gpu[done:done + len(a)] = (a + f) * 1e-3
            done += len(a)
    total = D.max(time.perf_counter() - t0)
    eng.set_timing(0)
    pc1 = eng.path_counters()
    paths = {k: pc1[k] - pc0[k] for k in pc1}
    # the last BAM's table against the one-shot counted table of the same BAMs: integer fields exact, GL / QUAL within
    # 1e-9 relative (the incremental folds add the fp64 sums in another grouping)
    same = None
    if nb == len(data):
        same = len(calls) == len(final_calls) and all(
            np.array_equal(calls[f], final_calls[f]) for f in ("pos", "dp", "ad", "pl", "score", "ref", "alt", "rank",
                                                                "first_batch", "gl_zero")) and all(
            np.allclose(calls[f], final_calls[f], rtol=1e-9, atol=0.0) for f in ("gl", "qual"))
    E_b = data.n_entries[:nb].astype(np.float64)
    # bytes per BAM the finalize path must move: the new BAM's base_code + qual + offsets (counted), the per-position
    # totals and REF chars the listing reads (2 x u32 + 1 B), the calls written
    moved = 2 * E_b + 8 * (C + 1) + 9 * C + 56 * n_calls
    g = gpu[:done]
    return {"bams": nb, "total_s": total, "ms_per_bam": total / nb * 1e3,
            "latency_ms_p50": float(np.median(lat)) * 1e3, "latency_ms_p99": float(np.percentile(lat, 99)) * 1e3,
            "latency_ms_first_100": float(np.mean(lat[:100])) * 1e3, "latency_ms_last_100": float(np.mean(lat[-100:])) * 1e3,
            "gpu_ms_per_bam": float(np.mean(g)) * 1e3, "gpu_ms_last_100": float(np.mean(g[-100:])) * 1e3,
            "bams_per_s": nb / total, "calls_last": int(n_calls[-1]), "final_table_equals_one_shot": same,
            "path": "per BAM: spg_accumulate_batches (1 borrowed batch) + spg_finalize (counted mode from BAM 1: "
                    "k_acc_lite_run over the new BAM, k_count_list, incremental k_fold_hist, sparse k_finalize) + "
                    "spg_get_candidates",
            "engine_paths": paths,
            "roofline": {"bound": "hbm (launch-bound at 6 MB per BAM)", "achieved": float(np.mean(moved[:done]) / np.mean(g) / 1e9),
                         "peak": PEAK_HBM / 1e9, "unit": "GB/s",
                         "frac": float(np.mean(moved[:done]) / np.mean(g) / PEAK_HBM),
                         "algorithmic_bytes_per_bam": float(np.mean(moved))}}


def cpu_model():
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line.startswith("Model name:"):
                return line.split(":", 1)[1].strip()
    except (OSError, subprocess.SubprocessError):
        pass
    return None


def cpu_baseline(args):
    """Oracle restatements of the reference path on a bounded sample of the same workload, on this
    box's host cores: the Python/numpy port (1 core), the C restatement on 1 core and on every core
    this process may use (OpenMP)."""
    from covid_spings_variant_caller_amd import synth
    from oracle import reference_port as rp
    from oracle.c_oracle import COracle
    Lw, depth = args.eff_L, args.eff_depth
    ref = synth.reference(min(Lw, 10_000_000), seed=1)
    lo = 8000
    n = int(min(max(args.cpu_positions * 10000.0 / depth, 100), len(ref) - lo))
    _, off, c, q = synth.pileup(len(ref), depth, seed=2, ref=ref, lo=lo, hi=lo + n, max_depth=args.max_depth)
    t0 = time.perf_counter()
    o = rp.OracleCaller(ref, 30, 10, 5, 0.10)
    o.accumulate(lo, off, c, q)
    o.prepare_variants()
    t_py = time.perf_counter() - t0
    n_c = min(len(ref), max(n, int(3e8 / depth)))   # the C restatement: ~3e8 entries (the whole SARS genome)
    _, off2, c2, q2 = synth.pileup(len(ref), depth, seed=2, ref=ref, hi=n_c, max_depth=args.max_depth)
    res = {}
    cores = len(os.sched_getaffinity(0))
    # the multi-threaded leg runs on this process's CPU share: OMP_NUM_THREADS (16 per GPU on the pool's boxes,
    # whose affinity mask lists the whole machine) or, unset, every CPU in the affinity mask
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    share = min(cores, omp) if omp else cores
    for tag, threads in (("c_restatement", 1), (f"c_restatement_{share}_threads", share)):
        COracle.set_threads(threads)
        t0 = time.perf_counter()
        co = COracle(ref, 30, 10, 5, 0.10)
        co.accumulate(0, off2, c2, q2)
        co.finalize()
        t_c = time.perf_counter() - t0
        res[tag] = {"value": n_c / t_c, "unit": "positions/s", "cores": threads,
                    "sample": f"oracle/spg_oracle.c ({'OpenMP' if threads > 1 else 'sequential'}) on {n_c} positions "
                              f"({int(off2[-1])} entries), {t_c:.2f} s"}
        del co
    COracle.set_threads(1)
    return {"value": n / t_py, "unit": "positions/s", "cores": 1, "kind": "port",
            "sample": f"oracle/reference_port.py (Python/numpy restatement of live_variant_caller.py:74-185) "
                      f"on {n} positions x {depth:.0f}x ({int(off[-1])} entries), {t_py:.2f} s, 1 core; "
                      f"pysam pileup/BAM decode not included (absent)",
            **res, "cores_in_affinity_mask": cores, "omp_num_threads": omp or None, "cpu_model": cpu_model()}


def vcqueue_loop(caller, paths, work_dir):
    """client_server/vc_queue.py:134-144 per BAM, in its order and with its file names: process_bam, then
    create_checkpoint(<temp dir>/<bam name>.pkl), then write_vcf(<output dir>/<bam name>.vcf) — per-stage wall time
    (the GPU work included: write_vcf's prepare_variants reads the call table back)."""
    import contextlib
    import io
    tmp = os.path.join(work_dir, "vcq_tmp")
    out = os.path.join(work_dir, "vcq_out")
    os.makedirs(tmp, exist_ok=True)
    os.makedirs(out, exist_ok=True)
    caller.reset_memory()
    caller.engine.sync()
    st = np.zeros((len(paths), 3))
    t_all = time.perf_counter()
    for k, p in enumerate(paths):
        name = os.path.basename(p)
        t0 = time.perf_counter()
        caller.process_bam(p)
        t1 = time.perf_counter()
        caller.create_checkpoint(os.path.join(tmp, name + ".pkl"))
        t2 = time.perf_counter()
        with contextlib.redirect_stdout(io.StringIO()):          # (write_vcf prints the path, :234)
            caller.write_vcf(os.path.join(out, name + ".vcf"))
        t3 = time.perf_counter()
        st[k] = (t1 - t0, t2 - t1, t3 - t2)
    caller.flush_checkpoints()                   # (write-behind: the last shard and manifest on disk, inside the timing)
    total = time.perf_counter() - t_all
    n_calls = sum(1 for ln in open(os.path.join(out, os.path.basename(paths[-1]) + ".vcf")) if not ln.startswith("#"))
    import shutil
    shutil.rmtree(tmp, ignore_errors=True)
    shutil.rmtree(out, ignore_errors=True)
    return {"bams": len(paths), "positions_per_s_per_bam": len(paths) * L_SARS / total, "ms_per_bam": total / len(paths) * 1e3,
            "process_bam_ms": float(st[:, 0].mean()) * 1e3, "create_checkpoint_ms": float(st[:, 1].mean()) * 1e3,
            "write_vcf_ms": float(st[:, 2].mean()) * 1e3,
            "per_bam_ms": [[round(x * 1e3, 2) for x in r] for r in st],
            "checkpoint_shard_mb": round(caller.last_checkpoint_bytes / 1e6, 2),
            "checkpoint_write_behind": caller.checkpoint_write_behind,
            "calls_last_vcf": n_calls, "bam_path": caller.last_bam_path,
            "path": "process_bam (BAM in HBM from 32 MiB files, else the records plan) -> create_checkpoint (this BAM's batch compacted and packed on the GPU "
                    "into pinned memory; a helper thread writes the shard, then the per-BAM manifest listing the memory's earlier shards, while the "
                    "next BAM runs) -> write_vcf (prepare_variants + VCF text); ms_per_bam includes the last checkpoint's write"}


def end_to_end(args, device):
    """BAM -> calls through the drop-in (LiveVariantCaller.process_bam, live_variant_caller.py:54-72).
    Product path (device pileup): host BGZF inflate straight into pinned memory + record scan +
    htslib depth cap / overlap tweak + CSR offsets (spp_pileup_plan_records) -> async H2D of the inflated BAM
    on the engine's copy stream -> k_pileup_fill decodes the records and walks the CIGARs -> accumulate; the
    next BAM's host work overlaps the previous BAM's copy and kernels.  Beside it, r02's host-fill path
    (the host writes every entry into pinned staging).  A stream of --e2e-bams synthetic
    10,000x BAMs (written by the C++ read simulator) into one memory, then prepare_variants.  Reported
    beside `value` (never as it): it includes the host front end and PCIe."""
    import tempfile
    from covid_spings_variant_caller_amd import synth
    from covid_spings_variant_caller_amd.live_variant_caller import LiveVariantCaller
    from covid_spings_variant_caller_amd.pileup import AlignmentFile, PileupParams, simulate_bam
    from covid_spings_variant_caller_amd.engine import pinned_empty
    ref = synth.reference(L_SARS, seed=1)
    d = tempfile.mkdtemp(dir=os.environ.get("TMPDIR", "/tmp"))
    bam = os.path.join(d, "sars_e2e.bam")
    fasta = os.path.join(d, "ref.fa")
    with open(fasta, "w") as f:
        f.write(">NC_045512.2\n")
        for i in range(0, L_SARS, 60):
            f.write(ref[i:i + 60] + "\n")
    t0 = time.perf_counter()
    n_reads = simulate_bam(bam, "NC_045512.2", ref, depth=args.eff_depth, seed=5, n_threads=args.e2e_threads)
    t_sim = time.perf_counter() - t0
    res = {}
    n_bams = max(1, args.e2e_bams)
    def stream(cap, mode):
        caller = LiveVariantCaller(fasta, 30, 20, 10, 5, 0.10, 1, device=device, max_depth=cap,
                                   n_threads=args.e2e_threads, pileup=mode)
        for _ in range(3):                         # warm-up: pinned staging / record buffers, library state
            caller.process_bam(bam)
        assert caller.last_bam_path == mode, (caller.last_bam_path, mode)
        caller.reset_memory()
        caller.engine.sync()
        t0 = time.perf_counter()
        for _ in range(n_bams):
            caller.process_bam(bam)
        t_in = time.perf_counter() - t0
        calls = caller.prepare_variants()
        caller.engine.sync()
        t1 = time.perf_counter()
        return caller, calls, t0, t_in, t1

    def device_breakdown_gpu_plan(caller, reps=3):
        """One BAM through the product's device path (r06): the depth cap and mate pairing on the GPU
        (spg_bam_plan_build) — nothing comes down; each stage synchronised."""
        eng, prm = caller.engine, caller.pileup_params
        rows = []
        for _ in range(reps):
            eng.reset()
            eng.sync()
            t = [time.perf_counter()]
            with AlignmentFile(bam) as f:
                tid = f.tid("NC_045512.2")
                m = f.bam_map(prm.n_threads)
                t.append(time.perf_counter())
                n = eng.bam_open(m, tid, prm)
                m.close()
                t.append(time.perf_counter())
                plan = eng.bam_plan_build(prm.max_depth, prm.ignore_overlaps)
                assert plan is not None, eng.bam_fallback
                t.append(time.perf_counter())
            assert eng.bam_accumulate_planned(plan)
            eng.wait_input()
            eng.sync()
            t.append(time.perf_counter())
            eng.finalize()
            eng.sync()
            t.append(time.perf_counter())
            rows.append(np.diff(t) * 1e3)
        r = np.median(np.array(rows), axis=0)
        return {"map_and_pinned_copy_ms": r[0], "bam_open_ms (H2D + inflate + CRC + record scan + fields)": r[1],
                "inflate_kernels_ms": eng.bam_inflate_ms(), "gpu_depth_cap_and_pairing_ms": r[2],
                "tweak_fill_ms": r[3], "finalize_ms": r[4], "reads": int(n), "pairs": int(plan.n_pairs),
                "sum_ms": float(r.sum())}

    def device_breakdown(caller, reps=3):
        """One BAM through the device path's stages with the host plan (r05's product path: fields down, the depth
        cap / pairing replayed on the host, the plan up), each synchronised (their sum exceeds the pipelined per-BAM
        time: process_bam returns once the fill is enqueued)."""
        eng, prm = caller.engine, caller.pileup_params
        rows = []
        for _ in range(reps):
            eng.reset()
            eng.sync()
            t = [time.perf_counter()]
            with AlignmentFile(bam) as f:
                tid = f.tid("NC_045512.2")
                m = f.bam_map(prm.n_threads)
                t.append(time.perf_counter())
                n = eng.bam_open(m, tid, prm)
                m.close()
                t.append(time.perf_counter())
                reads = eng.bam_reads(n)
                t.append(time.perf_counter())
                pb = f.pileup_fields("NC_045512.2", reads, prm)
                t.append(time.perf_counter())
            assert eng.bam_accumulate(pb)
            eng.wait_input()
            eng.sync()
            t.append(time.perf_counter())
            eng.finalize()
            eng.sync()
            t.append(time.perf_counter())
            pb.close()
            rows.append(np.diff(t) * 1e3)
        r = np.median(np.array(rows), axis=0)
        return {"map_and_pinned_copy_ms": r[0], "bam_open_ms (H2D + inflate + CRC + record scan + fields)": r[1],
                "inflate_kernels_ms": eng.bam_inflate_ms(), "reads_fields_d2h_ms": r[2],
                "host_depth_cap_and_pairing_ms": r[3], "plan_h2d_tweak_fill_ms": r[4], "finalize_ms": r[5],
                "reads": int(n), "sum_ms": float(r.sum())}

    for cap, tag in ((8000, "parity_mode_max_depth_8000"), (0, "uncapped")):
        # the host-fill path first (r02's product path: the host writes every entry into pinned staging)
        caller, calls_h, t0, t_in, t1 = stream(cap, "host")
        host_leg = {"positions_per_s_per_bam": n_bams * L_SARS / (t1 - t0), "s_per_bam": (t1 - t0) / n_bams}
        caller.engine.close()
        del caller
        # r03-r04's product path: the host plans the records (GPU inflate), the GPU writes the entries
        caller, calls_r, t0, t_in, t1 = stream(cap, "records")
        assert [v["start"] for v in calls_r] == [v["start"] for v in calls_h], "records / host pileup calls differ"
        rec_leg = {"positions_per_s_per_bam": n_bams * L_SARS / (t1 - t0), "s_per_bam": (t1 - t0) / n_bams}
        p = caller.pileup_params
        b0 = time.perf_counter()
        with AlignmentFile(bam) as f:
            b = f.pileup_records("NC_045512.2", p)
        b1 = time.perf_counter()
        rec_leg["host_plan_records_s"] = b1 - b0
        rec_leg["inflated_mb"] = b.records().data_bytes / 1e6
        b.close()
        caller.engine.close()
        del caller
        # the product path: the BAM kept in HBM (spg_bam_*)
        caller, calls, t0, t_in, t1 = stream(cap, "device")
        assert [v["start"] for v in calls] == [v["start"] for v in calls_h], "device / host pileup calls differ"
        brk = device_breakdown_gpu_plan(caller)
        brk_host = device_breakdown(caller)
        # the same BAMs through process_bams (the drop-in's many-BAM call: the BAM-in-HBM path pipelined over two device
        # BAM slots, the next BAM opening on the GPU while the host plans this one); a warm-up call first (device buffers)
        caller.process_bams([bam] * 2)
        caller.reset_memory()
        caller.engine.sync()
        m0 = time.perf_counter()
        caller.process_bams([bam] * (2 * n_bams))
        calls_m = caller.prepare_variants()
        caller.engine.sync()
        m1 = time.perf_counter()
        assert [v["start"] for v in calls_m] == [v["start"] for v in calls_h], "process_bams calls differ"
        # vc_queue.py:134-144's loop over BAM files with their own names (hard links of the simulated BAM)
        vq = []
        for k in range(max(2, n_bams)):
            pth = os.path.join(d, f"vq{k}.bam")
            os.link(bam, pth)
            vq.append(pth)
        vq_leg = vcqueue_loop(caller, vq, d)
        caller.checkpoint_write_behind = True            # the same loop with write-behind checkpoints (opt-in)
        vq_leg_wb = vcqueue_loop(caller, vq, d)
        caller.checkpoint_write_behind = False
        for pth in vq:
            os.remove(pth)
        many_leg = {"bams": 2 * n_bams, "positions_per_s_per_bam": 2 * n_bams * L_SARS / (m1 - m0),
                    "s_per_bam": (m1 - m0) / (2 * n_bams),
                    "path": ("BAMs kept in HBM, pipelined over two device BAM slots (spg_bam_slot): BAM i + 1 opens on "
                             "the GPU while the host plans BAM i" if caller.last_bam_path == "device" else
                             "records plans (two at once on the host threads), BGZF inflate " +
                             ("on the GPU (spg_bgzf_inflate)" if caller.last_gpu_inflate else "on the host"))}
        res[tag] = {"bams": n_bams, "positions_per_s_per_bam": n_bams * L_SARS / (t1 - t0),
                    "s_per_bam": (t1 - t0) / n_bams, "ingest_s": t_in, "finalize_s": t1 - t0 - t_in,
                    "calls": len(calls), "reads_per_bam": int(brk["reads"]),
                    "path": "BAM kept in HBM (process_bam, pileup='device'): compressed file H2D -> k_inflate_par + k_crc32 "
                            "-> record scan + stepper filter + fields on the GPU -> depth cap / mate pairing on the GPU "
                            "(spg_bam_plan_build: k_plan_sweep + name-group replay) -> mate-overlap tweak + k_pileup_fill "
                            "-> accumulate",
                    "breakdown_one_bam_device": brk, "breakdown_one_bam_host_plan": brk_host,
                    "plan_path": caller.last_plan_path,
                    "records_plan_path": rec_leg, "host_fill_path": host_leg, "process_bams": many_leg,
                    "vcqueue_loop": vq_leg, "vcqueue_loop_write_behind": vq_leg_wb}
        caller.engine.close()
        del caller
    res["bam_bytes"] = os.path.getsize(bam)
    res["reads"] = n_reads
    res["simulate_s"] = t_sim
    res["host_threads"] = args.e2e_threads
    from covid_spings_variant_caller_amd import _native as N
    res["host_inflater"] = N.pileup_lib().spp_host_inflater().decode()     # (records plans / host fills)
    os.remove(bam)
    if args.e2e_many > 0:
        # BASELINE config 4 from files: many 100x BAMs through LiveVariantCaller.process_bams (plans on a thread
        # pool, per-BAM batches accumulated in order, counted at prepare_variants)
        paths = []
        t0 = time.perf_counter()
        for i in range(args.e2e_many):
            pth = os.path.join(d, f"m{i}.bam")
            simulate_bam(pth, "NC_045512.2", ref, depth=100.0, seed=1000 + i, n_threads=args.e2e_threads)
            paths.append(pth)
        t_sim = time.perf_counter() - t0
        caller = LiveVariantCaller(fasta, 30, 20, 10, 5, 0.10, 1, device=device, max_depth=8000,
                                   n_threads=args.e2e_threads)
        caller.process_bams(paths[:4])                # warm-up
        caller.reset_memory()
        caller.engine.sync()
        t0 = time.perf_counter()
        caller.process_bams(paths)
        t_in = time.perf_counter() - t0
        calls = caller.prepare_variants()
        caller.engine.sync()
        t1 = time.perf_counter()
        vq_many = vcqueue_loop(caller, paths[:16], d)
        res["config4_process_bams"] = {
            "bams": len(paths), "depth": 100, "positions_per_s": len(paths) * L_SARS / (t1 - t0),
            "s_per_bam": (t1 - t0) / len(paths), "ingest_s": t_in, "prepare_variants_s": t1 - t0 - t_in,
            "calls": len(calls), "bam_bytes_each": os.path.getsize(paths[0]), "simulate_s": t_sim,
            "path": "process_bams: host plans on a thread pool -> pinned staging -> per-BAM batches -> "
                    "counted mode (k_acc_lite_run + k_count_list + k_fold_hist) + sparse finalize",
            "vcqueue_loop": vq_many}
        caller.engine.close()
        del caller
        for pth in paths:
            os.remove(pth)
    os.remove(fasta)
    os.rmdir(d)
    return res


LINE_LIMIT = 4096      # bytes of the printed line (the driver parses the tail of stdout: r05's 20.5 KB line was lost)
HEAD_KEYS = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
             "vs_baseline", "dtype", "data")


def _r(x, nd=4):
    """A number rounded to nd significant digits (the compact line carries no 17-digit floats)."""
    if isinstance(x, float) and math.isfinite(x) and x != 0.0:
        return float(f"{x:.{nd}g}")
    return x


def _leg(d, frac=True):
    """{value, ms_per_step, frac} of one nested leg (None entries dropped)."""
    if not isinstance(d, dict):
        return None
    if "error" in d:
        return {"error": str(d["error"])[:160]}
    out = {"value": _r(d.get("value")), "ms_per_step": _r(d.get("ms_per_step"))}
    if frac and isinstance(d.get("roofline"), dict):
        out["frac"] = _r(d["roofline"].get("frac"), 3)
    return {k: v for k, v in out.items() if v is not None}


def _e2e(e):
    """The end-to-end leg in a few numbers: positions/s per 10,000x BAM through the lone process_bam, process_bams, and
    the VCQueue loop's ms per BAM (uncapped / max_depth 8000)."""
    out = {}
    for tag, key in (("uncapped", "uncapped"), ("capped", "parity_mode_max_depth_8000")):
        s = e.get(key)
        if not isinstance(s, dict):
            continue
        o = {"process_bam_pos_s": _r(s.get("positions_per_s_per_bam"))}
        if isinstance(s.get("process_bams"), dict):
            o["process_bams_pos_s"] = _r(s["process_bams"].get("positions_per_s_per_bam"))
        if isinstance(s.get("vcqueue_loop"), dict):
            o["vcqueue_ms_per_bam"] = _r(s["vcqueue_loop"].get("ms_per_bam"))
        b = s.get("breakdown_one_bam_device")
        if isinstance(b, dict):
            o["gpu_cap_pairing_ms"] = _r(b.get("gpu_depth_cap_and_pairing_ms"), 3)
            o["inflate_ms"] = _r(b.get("inflate_kernels_ms"), 3)
        b = s.get("breakdown_one_bam_host_plan")
        if isinstance(b, dict):
            o["host_cap_pairing_ms"] = _r(b.get("host_depth_cap_and_pairing_ms"), 3)
        out[tag] = o
    if "host_inflater" in e:
        out["host_inflater"] = e["host_inflater"]
    c4 = e.get("config4_process_bams")
    if isinstance(c4, dict):
        out["config4_process_bams_pos_s"] = _r(c4.get("positions_per_s"))
    return out


def compact_line(res):
    """The one JSON line rank 0 prints: the contract's headline keys, `config`, `roofline` (without prose), a compact
    `cpu_baseline`, and {value, ms_per_step, frac} per nested leg — under LINE_LIMIT bytes.  Everything else (per-
    measurement times, breakdowns, per-BAM arrays, the multi-device detail) goes to the detail file (`detail`)."""
    line = {k: res[k] for k in HEAD_KEYS if k in res}
    for k in ("value", "ms_per_step"):
        if isinstance(line.get(k), float):
            line[k] = float(f"{line[k]:.6g}")
    cfg = dict(res.get("config", {}))
    if isinstance(cfg.get("ranks"), list):
        cfg["ranks"] = len(cfg["ranks"])
    line["config"] = cfg
    tm = res.get("timing")
    if isinstance(tm, dict):
        line["timing"] = {k: tm[k] for k in ("measurements", "steps_per_measurement") if k in tm}
    rf = res.get("roofline")
    if isinstance(rf, dict):
        line["roofline"] = {k: _r(rf[k], 5) for k in ("bound", "achieved", "peak", "unit", "frac", "traffic",
                                                       "traffic_source", "kernel", "kernel_ms", "algorithmic_bytes")
                            if k in rf}
    cb = res.get("cpu_baseline")
    if isinstance(cb, dict):
        line["cpu_baseline"] = {k: _r(cb[k]) for k in ("value", "unit", "cores", "kind") if k in cb}
        line["cpu_baseline"]["sample"] = str(cb.get("sample", ""))[:200]
        for k in ("c_restatement", "c_restatement_16_threads"):
            if isinstance(cb.get(k), dict):
                line["cpu_baseline"][k] = {"value": _r(cb[k].get("value")), "cores": cb[k].get("cores")}
    legs = {}
    for k in ("parity_mode", "sars1k", "sars100k", "chr1_30x", "multi_device"):
        if k in res:
            legs[k] = _leg(res[k])
    if isinstance(res.get("sars100k"), dict) and "parity_mode" in res["sars100k"]:
        legs["sars100k_capped"] = _leg(res["sars100k"]["parity_mode"])
    if isinstance(res.get("config4"), dict):
        legs["config4"] = _leg(res["config4"])
        pb = res["config4"].get("per_bam_finalize")
        if isinstance(pb, dict):
            legs["config4_per_bam_finalize"] = {"ms_per_bam": _r(pb.get("ms_per_bam"))}
    if isinstance(res.get("end_to_end"), dict):
        legs["end_to_end"] = _e2e(res["end_to_end"])
    if legs:
        line["legs"] = legs
    if "detail" in res:
        line["detail"] = res["detail"]
    s = json.dumps(line)
    if len(s) > LINE_LIMIT:                      # (never expected: drop the legs before the headline)
        line.pop("legs", None)
        line["legs_dropped"] = "line limit"
    return line


def emit(res, detail_out):
    """Write the full nested result to `detail_out` (when it can be written) and print the compact line."""
    if detail_out:
        detail_out = detail_out.format(n=res.get("n_gpus", 1))
        try:
            os.makedirs(os.path.dirname(os.path.abspath(detail_out)), exist_ok=True)
            with open(detail_out, "w") as f:
                json.dump(res, f)
            res = dict(res, detail=os.path.relpath(os.path.abspath(detail_out), ROOT))
        except OSError as e:
            print(f"bench: detail file {detail_out}: {e}", file=sys.stderr)
    print(json.dumps(compact_line(res)), flush=True)


def main():
    args = parse()
    legs = set() if args.legs == "none" else set(args.legs.split(","))
    if args.no_parity: legs.discard("parity")
    if args.no_chr1: legs.discard("chr1")
    if args.no_e2e: legs.discard("e2e")
    if args.no_cpu_baseline: legs.discard("cpu")
    if args.many_batches <= 0 and args.runs_batches <= 0: legs.discard("config4")
    if args.multi_helper:
        sys.exit(multi_helper(args))
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # no launcher: one rank process per GPU, started before anything here touches a GPU
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    world0 = int(os.environ.get("WORLD_SIZE", "1"))
    helper = None
    if world0 > 1 and int(os.environ.get("RANK", "0")) == 0 and not args.no_main and args.workload != "sars_many":
        # rank 0's helper for the multi-device leg, started before this process touches a GPU (it waits for a line on
        # its stdin before it does): RCCL's one-process init over every device then runs in a process that rank 0 can
        # stop after a time limit, and a hang there cannot take the per-rank line with it
        helper = subprocess.Popen([sys.executable, os.path.abspath(__file__), "--multi-helper"] + sys.argv[1:],
                                  stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
    import torch
    import spings  # noqa: F401
    if not args.e2e_threads:
        from covid_spings_variant_caller_amd.pileup import cpu_share
        args.e2e_threads = max(1, min(len(os.sched_getaffinity(0)) // 8, cpu_share()))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world and rank == 0:
        print(f"bench: --gpus {args.gpus} but WORLD_SIZE {world}: timing {world} rank(s)", file=sys.stderr)
    if args.backend != "nccl":                  # functional runs of the N > 1 path on fewer GPUs
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    D = Dist(world, rank, args.backend, torch.device("cuda", local))
    props = torch.cuda.get_device_properties(local)
    rank_devices = D.all_gather_object({"rank": rank, "device": local, "pci_bus_id": getattr(props, "pci_bus_id", None),
                                        "name": props.name})

    if args.workload == "sars_many":
        c4 = run_config4(args, D, local, world, rank)
        res = {"metric": "pileup positions/s, BASELINE config 4 (BAMs x positions accumulated per second)",
               "value": c4["value"], "unit": "positions/s", "n_gpus": world, "steps": c4["steps"],
               "warmup": args.warmup, "ms_per_step": c4["ms_per_step"], "higher_is_better": True,
               "scaling": "strong", "vs_baseline": None, "dtype": "u8/f64", "data": "synthetic",
               "config": {"workload": c4["workload"], "parallelism": f"coord-shard x{world}"}, **c4}
        if rank == 0:
            emit(res, args.detail_out)
        D.close()
        return
    L, depth, contig = WORKLOADS[args.workload]
    L = args.length or L
    depth = args.depth or depth
    args.eff_L, args.eff_depth = L, depth
    if args.no_main:                            # (profiling: one nested leg on its own)
        args.steps, args.reps, args.warmup = max(1, args.steps), max(1, args.reps), max(0, args.warmup)
        main_pt = {"E": 0, "C": 0, "value": None, "steps": 0, "reps": 0, "ms_per_step": None, "achieved": 0.0,
                   "kernel_ms": None, "kernel_ms_median": None, "kernel_samples": 0, "algo_bytes": 0,
                   "measurements_ms": [], "finalize_ms": None, "host_enqueue_ms_per_step": None, "n_cand": 0,
                   "n_replay": 0, "t_gen": 0.0, "gathered": None}
    else:
        main_pt = run_point(args, D, L, depth, args.max_depth, local, world, rank, contig)
    E, C = main_pt["E"], main_pt["C"]
    res = {
        "metric": ("pileup positions/s at 10,000x depth (SARS-CoV-2, synthetic)" if args.workload == "sars10k"
                   and depth == 10000 and L == L_SARS else f"pileup positions/s at {depth:,.0f}x depth ({contig} "
                   f"L={L:,}, synthetic)"),
        "value": main_pt["value"], "unit": "positions/s", "n_gpus": world, "steps": main_pt["steps"],
        "warmup": args.warmup, "ms_per_step": main_pt["ms_per_step"], "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8/f64", "data": "synthetic",
        "config": {"workload": f"{args.workload}: {contig} L={L}, {depth:.0f}x, 150-bp reads, "
                               + ("uncapped" if not args.max_depth else f"max_depth {args.max_depth}")
                               + ", 1 sample per GPU per step (coordinate-sharded)",
                   "positions_per_step": world * L, "entries_per_gpu_step": E, "columns_per_gpu": C,
                   "parallelism": f"coord-shard x{world}",
                   "ranks": rank_devices,
                   "collective": (f"torch.distributed {args.backend} ({'RCCL over xGMI' if args.backend == 'nccl' else 'host'}) "
                                  f"gather of the call tables to rank 0, one per step" if world > 1 else "none (N = 1)"),
                   "engine_mode": "full_table" if args.full_table else "calls_only"},
        "timing": {"measurements": len(main_pt["measurements_ms"]), "steps_per_measurement": main_pt["steps"],
                   "steps_timed_total": main_pt["steps"] * main_pt["reps"],
                   "steps_requested": args.steps, "measurement_ms": main_pt["measurements_ms"],
                   "statistic": "median of --reps measurements, each exactly `steps` back-to-back steps between "
                                "barrier + device synchronize (--min-ms 0); max over ranks"},
        "roofline": {"bound": "hbm", "achieved": main_pt["achieved"] / 1e9, "peak": PEAK_HBM / 1e9, "unit": "GB/s",
                     "frac": main_pt["achieved"] / PEAK_HBM,
                     "traffic": pmc_traffic(kernel_name(E, C, not args.full_table)[1], E),
                     "traffic_source": pmc_traffic(kernel_name(E, C, not args.full_table)[1], E, True)[1],
                     "traffic_note": TRAFFIC_NOTE,
                     "kernel": kernel_name(E, C, not args.full_table)[0], "kernel_ms": main_pt["kernel_ms"],
                     "kernel_ms_median": main_pt["kernel_ms_median"], "kernel_samples": main_pt["kernel_samples"],
                     "algorithmic_bytes": main_pt["algo_bytes"]},
        "finalize_ms": main_pt["finalize_ms"], "host_enqueue_ms_per_step": main_pt["host_enqueue_ms_per_step"],
        "candidates_per_gpu_step": main_pt["n_cand"],
        "replayed_positions_per_gpu_step": main_pt["n_replay"], "datagen_s": main_pt["t_gen"],
        "calls_gathered_per_step": main_pt["gathered"] if main_pt["gathered"] is not None else main_pt["n_cand"],
    }
    nested = args.workload == "sars10k" and not args.length and not args.depth
    if "parity" in legs and not args.max_depth and nested:
        res["parity_mode"] = nested_point(args, D, "sars10k", local, world, rank, max_depth=8000)
    if "sars1k" in legs and nested:           # BASELINE config 2
        res["sars1k"] = nested_point(args, D, "sars1k", local, world, rank, samples=args.sars1k_samples,
                                     distinct=min(16, args.sars1k_samples * world))
    if "sars100k" in legs and nested:         # BASELINE config 3, uncapped (the deep-column stress) and pysam's cap
        res["sars100k"] = nested_point(args, D, "sars100k", local, world, rank)
    if "sars100k_capped" in legs and nested:
        res.setdefault("sars100k", {})["parity_mode"] = nested_point(args, D, "sars100k", local, world, rank, max_depth=8000)
    if "config4" in legs and nested:          # BASELINE config 4
        res["config4"] = run_config4(args, D, local, world, rank)
    if "chr1" in legs and nested:             # BASELINE config 5
        res["chr1_30x"] = nested_point(args, D, "chr1_30x", local, world, rank, step_frac=True)
    if ("multi" in legs or world > 1) and not args.no_main and args.workload != "sars_many":
        # the drop-in's one-process multi-GPU path over devices 0..N-1 (always with N > 1), on rank 0 while the other
        # ranks wait on the host
        D.host_barrier()
        if rank == 0:
            if helper is not None:
                res["multi_device"] = run_helper(helper, args.multi_timeout)
                helper = None
            else:
                try:
                    res["multi_device"] = run_multi_device(args, world, L, depth, args.max_depth)
                except Exception as e:        # (reported, never fatal to the per-rank line)
                    res["multi_device"] = {"error": f"{type(e).__name__}: {e}"}
        D.host_barrier()
    if helper is not None:                        # (the leg did not run: let the helper go)
        helper.stdin.close()
        helper.wait(timeout=30)
    if rank == 0 and world == 1 and "e2e" in legs and L == L_SARS:
        res["end_to_end"] = end_to_end(args, 0)
    if rank == 0 and world == 1 and "cpu" in legs:
        res["cpu_baseline"] = cpu_baseline(args)
    if rank == 0:
        emit(res, args.detail_out)
    D.close()


if __name__ == "__main__":
    main()
