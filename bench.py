"""Benchmark: pileup positions/s at 10,000x depth on 1..8 MI355X (BASELINE.json metric).

One step = one pass of the hot path over one batch: reset the accumulators (new sample), accumulate
the batch's CSR pileup (HBM-resident, borrowed), finalize (per-position table + call table), and —
for N > 1 — gather the call tables to rank 0 over RCCL.  Workload (BASELINE config 2/"metric
point"): synthetic SARS-CoV-2 reference (L = 29,903), 10,000x depth, 150-bp reads, uncapped
(max_depth 0).  Weak scaling: with N GPUs a step processes N samples; rank r owns the r-th
coordinate range of every sample (one engine over the concatenated shards).

Timing: W untimed warm-up steps, then K steps between barrier + device synchronize; max over
ranks.  The dominant kernel's duration is measured with HIP events on the engine's stream.
"""
from __future__ import annotations

import argparse
import json
import os
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
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--workload", default="sars10k", choices=sorted(WORKLOADS) if False else
                    ["sars10k", "sars1k", "sars100k", "chr1_30x"])
    ap.add_argument("--depth", type=float, default=0.0, help="override the workload's depth")
    ap.add_argument("--length", type=int, default=0, help="override the workload's reference length")
    ap.add_argument("--max-depth", type=int, default=0, help="0 = uncapped; 8000 = pysam parity cap")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-positions", type=int, default=8000)
    ap.add_argument("--no-e2e", action="store_true", help="skip the end-to-end BAM -> calls leg")
    ap.add_argument("--time-every", type=int, default=8,
                    help="HIP events around the accumulate kernel on every K-th timed step (each event "
                         "pair idles the GPU for microseconds; 1 = every step)")
    ap.add_argument("--e2e-threads", type=int, default=16)
    ap.add_argument("--full-table", action="store_true", help="also accumulate every table GL term")
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend for N > 1 (nccl = RCCL; "
                                                      "gloo only to exercise the path on one GPU)")
    return ap.parse_args()


WORKLOADS = {   # BASELINE.json configs (the metric is quoted on sars10k; the others are optional runs)
    "sars10k": (L_SARS, 10000.0, "NC_045512.2"),
    "sars1k": (L_SARS, 1000.0, "NC_045512.2"),
    "sars100k": (L_SARS, 100000.0, "NC_045512.2"),
    "chr1_30x": (248956422, 30.0, "chr1"),
}


def build_shard(rank, world, L, depth, max_depth, device):
    """This rank's coordinate range of each of `world` samples, generated natively
    (libspings_pileup spp_synth_batch: SURVEY §8 d read model) and concatenated in HBM."""
    import torch
    from covid_spings_variant_caller_amd import synth
    from covid_spings_variant_caller_amd.pileup import synth_batch
    ref = synth.reference(L, seed=1)
    shard = (L + world - 1) // world
    lo, hi = rank * shard, min(L, (rank + 1) * shard)
    offs, dc, dq, refs = [np.zeros(1, np.uint64)], [], [], []
    base = 0
    threads = min(16, len(os.sched_getaffinity(0)))
    for s in range(world):
        b = synth_batch(ref, depth, lo=lo, hi=hi, seed=2 + s, n_threads=threads, max_depth=max_depth)
        offs.append(b.offsets[1:] + np.uint64(base))
        base += b.n_entries
        dc.append(torch.from_numpy(b.codes).to(device))
        dq.append(torch.from_numpy(b.quals).to(device))
        refs.append(ref[lo:hi])
        b.close()
    pad = torch.zeros(16, dtype=torch.uint8, device=device)
    d_c = torch.cat(dc + [pad + 0xFF])
    d_q = torch.cat(dq + [pad])
    off = np.concatenate(offs)
    d_off = torch.from_numpy(off.view(np.int64).copy()).to(device)
    return ref, "".join(refs), off, d_off, d_c, d_q, int(base)


def cpu_baseline(args):
    """Oracle restatements of the reference path on a bounded sample of the same workload."""
    from covid_spings_variant_caller_amd import synth
    from oracle import reference_port as rp
    from oracle.c_oracle import COracle
    Lw, depth = args.eff_L, args.eff_depth
    ref = synth.reference(min(Lw, 10_000_000), seed=1)
    lo = 8000
    # about 8e7 entries (~13 s in the numpy port) whatever the depth
    n = int(min(max(args.cpu_positions * 10000.0 / depth, 100), len(ref) - lo))
    _, off, c, q = synth.pileup(len(ref), depth, seed=2, ref=ref, lo=lo, hi=lo + n, max_depth=args.max_depth)
    t0 = time.perf_counter()
    o = rp.OracleCaller(ref, 30, 10, 5, 0.10)
    o.accumulate(lo, off, c, q)
    o.prepare_variants()
    t_py = time.perf_counter() - t0
    n_c = min(len(ref), max(n, int(3e8 / depth)))   # the C restatement: ~3e8 entries (the whole SARS genome)
    _, off2, c2, q2 = synth.pileup(len(ref), depth, seed=2, ref=ref, hi=n_c, max_depth=args.max_depth)
    t0 = time.perf_counter()
    co = COracle(ref, 30, 10, 5, 0.10)
    co.accumulate(0, off2, c2, q2)
    co.finalize()
    t_c = time.perf_counter() - t0
    return {"value": n / t_py, "unit": "positions/s", "cores": 1, "kind": "port",
            "sample": f"oracle/reference_port.py (Python/numpy restatement of live_variant_caller.py:74-185) "
                      f"on {n} positions x {depth:.0f}x ({int(off[-1])} entries), {t_py:.2f} s, 1 core; "
                      f"pysam pileup/BAM decode not included (absent)",
            "c_restatement": {"value": n_c / t_c, "unit": "positions/s", "cores": 1,
                              "sample": f"oracle/spg_oracle.c on {n_c} positions ({int(off2[-1])} entries), {t_c:.2f} s"}}


def end_to_end(args, device):
    """BAM -> host pileup (libspings_pileup: BGZF inflate, htslib-rule pileup, CSR) -> H2D ->
    accumulate -> finalize -> call table, on one synthetic 10,000x BAM written by the C++ read
    simulator.  Reported beside `value` (never as it): it includes the host front end and PCIe."""
    import tempfile
    from covid_spings_variant_caller_amd import synth
    from covid_spings_variant_caller_amd.engine import PileupEngine
    from covid_spings_variant_caller_amd.pileup import AlignmentFile, PileupParams, simulate_bam
    ref = synth.reference(L_SARS, seed=1)
    d = tempfile.mkdtemp(dir=os.environ.get("TMPDIR", "/tmp"))
    bam = os.path.join(d, "sars_e2e.bam")
    t0 = time.perf_counter()
    n_reads = simulate_bam(bam, "NC_045512.2", ref, depth=args.eff_depth, seed=5, n_threads=args.e2e_threads)
    t_sim = time.perf_counter() - t0
    eng = PileupEngine(L_SARS, 30, 10, 5, 0.10, device=device, reference=ref, calls_only=True)
    res = {}
    for cap, tag in ((8000, "parity_mode_max_depth_8000"), (0, "uncapped")):
        eng.reset()
        t0 = time.perf_counter()
        with AlignmentFile(bam) as f:
            b = f.pileup_batch("NC_045512.2", PileupParams(max_depth=cap, n_threads=args.e2e_threads))
        t1 = time.perf_counter()
        eng.accumulate(b.pos_begin, b.offsets, b.codes, b.quals)
        eng.finalize()
        n_calls = len(eng.candidates())
        t2 = time.perf_counter()
        res[tag] = {"positions_per_s": L_SARS / (t2 - t0), "host_pileup_s": t1 - t0, "h2d_gpu_s": t2 - t1,
                    "entries": int(b.n_entries), "reads_used": int(b.n_reads_used), "calls": n_calls,
                    "pcie_inclusive_gpu_positions_per_s": L_SARS / (t2 - t1)}
        b.close()
    eng.close()
    res["bam_bytes"] = os.path.getsize(bam)
    res["reads"] = n_reads
    res["simulate_s"] = t_sim
    res["host_threads"] = args.e2e_threads
    os.remove(bam)
    os.rmdir(d)
    return res


def kernel_name(E, C):
    """The accumulate instantiation launch_accumulate (csrc/spg_kernels.hip) picks for this batch."""
    if E < 256 * C:
        return "k_acc_shallow + k_acc_seg<1,true,4,false> (spg_accumulate)"
    nt = 2 * E > (192 << 20)
    return f"k_acc_seg<4,true,4,{'true' if nt else 'false'}> (spg_accumulate{'; non-temporal loads' if nt else ''})"


def pmc_traffic(E):
    """HBM bytes per launch of the accumulate kernel from the newest committed PMC summary
    (profiles/rNN_bench_pmc.json, written by tools/summarize_prof.py from rocprofv3 --pmc passes of
    this bench: FETCH_SIZE x2 + WRITE_SIZE), when it was measured on this workload; else None."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_bench_pmc.json")))
    if not files:
        return None
    try:
        d = json.load(open(files[-1]))
        rec = next((v for k, v in d.items() if k.startswith("spg::k_acc_seg<4, true")), None)
        if rec is None or rec.get("entries") != E:
            return None
        return rec.get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def main():
    args = parse()
    import torch
    import spings  # noqa: F401
    from covid_spings_variant_caller_amd import synth
    from covid_spings_variant_caller_amd.engine import PileupEngine

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.backend != "nccl":                  # functional runs of the N > 1 path on fewer GPUs
        local = local % max(1, torch.cuda.device_count())
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(args.backend)
    else:
        torch.cuda.set_device(0)

    L, depth, contig = WORKLOADS[args.workload]
    L = args.length or L
    depth = args.depth or depth
    args.eff_L, args.eff_depth = L, depth
    dev = torch.device("cuda", local if world > 1 else 0)
    t_gen = time.perf_counter()
    ref, vref, off, d_off, d_c, d_q, E = build_shard(rank, world, L, depth, args.max_depth, dev)
    C = len(off) - 1
    t_gen = time.perf_counter() - t_gen
    # calls-only engine (SPG_P_CALLS_ONLY): the call table prepare_variants() returns, exactly; see
    # DESIGN.md §3 — the per-position GL table's REF-major entries are not accumulated
    eng = PileupEngine(C, 30, 10, 5, 0.10, device=local if world > 1 else 0, reference=vref,
                       calls_only=not args.full_table)

    # call-table gather buffer: u64 count + records, sized from a first (untimed) pass so the
    # per-step gather moves KBs, not the engine's full candidate capacity
    eng.reset()
    eng.accumulate(0, d_off, d_c, d_q, borrow=True, n_entries=E)
    eng.finalize()
    cand_cap = max(64, 4 * eng.counts()[0])
    if dist is not None:
        t = torch.tensor([cand_cap], dtype=torch.int64, device=d_c.device if args.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        cand_cap = int(t.item())
    gather_buf = torch.zeros(cand_cap * 56 + 8, dtype=torch.uint8, device=d_c.device)
    gather_out = [torch.empty_like(gather_buf) for _ in range(world)] if rank == 0 else None

    def step():
        eng.reset()
        eng.accumulate(0, d_off, d_c, d_q, borrow=True, n_entries=E)
        eng.finalize()
        if dist is not None:
            eng.copy_candidates_device(gather_buf, cap=cand_cap)
            if args.backend == "nccl":
                dist.gather(gather_buf, gather_out, dst=0)           # RCCL over xGMI
            else:
                dist.gather(gather_buf.cpu(), [o.cpu() for o in gather_out] if rank == 0 else None, dst=0)

    for _ in range(args.warmup):
        step()
    eng.sync()
    eng.kernel_times()                   # drop the warm-up steps' timings
    # timed region: HIP events around the accumulate kernel on every time_every-th step (a uniform
    # sample of the timed steps; events on every step would idle the GPU between launches)
    eng.set_timing(0)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    every = max(1, args.time_every)
    for k in range(args.steps):
        eng.set_timing(1 if k % every == 0 else 0)
        step()
    eng.sync()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    dt = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([dt], dtype=torch.float64, device=d_c.device if args.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    acc_ms, _ = eng.kernel_times(max(256, args.steps))  # HIP events of the sampled timed steps
    acc_ms = acc_ms[acc_ms > 0]
    eng.set_timing(2)                    # finalize duration from a few extra (untimed) steps
    for _ in range(8):
        step()
    eng.sync()
    _, fin_ms = eng.kernel_times()
    n_cand, n_replay = eng.counts()
    gathered = None
    if dist is not None and rank == 0:
        gathered = [int(o[:8].cpu().numpy().view(np.uint64)[0]) for o in gather_out]
        if max(gathered) > cand_cap:
            raise RuntimeError(f"call table larger than the gather buffer ({max(gathered)} > {cand_cap})")
    positions_per_step = world * L
    value = positions_per_step * args.steps / dt
    t_acc = float(np.mean(acc_ms)) * 1e-3
    t_fin = float(np.mean(fin_ms)) * 1e-3
    algo_bytes = 2 * E + 8 * (C + 1)          # base_code + qual + u64 offsets read by the accumulate kernel
    achieved = algo_bytes / t_acc
    res = {
        "metric": ("pileup positions/s at 10,000x depth (SARS-CoV-2, synthetic)" if args.workload == "sars10k"
                   and depth == 10000 and L == L_SARS else f"pileup positions/s at {depth:,.0f}x depth ({contig} "
                   f"L={L:,}, synthetic)"),
        "value": value, "unit": "positions/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "u8/f64", "data": "synthetic",
        "config": {"workload": f"{args.workload}: {contig} L={L}, {depth:.0f}x, 150-bp reads, "
                               + ("uncapped" if not args.max_depth else f"max_depth {args.max_depth}")
                               + ", 1 sample per GPU per step (coordinate-sharded)",
                   "positions_per_step": positions_per_step, "entries_per_gpu_step": E, "columns_per_gpu": C,
                   "parallelism": f"coord-shard x{world}",
                   "engine_mode": "full_table" if args.full_table else "calls_only"},
        "roofline": {"bound": "hbm", "achieved": achieved / 1e9, "peak": PEAK_HBM / 1e9, "unit": "GB/s",
                     "frac": achieved / PEAK_HBM, "traffic": pmc_traffic(E),
                     "kernel": kernel_name(E, C), "kernel_ms": t_acc * 1e3, "algorithmic_bytes": algo_bytes},
        "finalize_ms": t_fin * 1e3, "candidates_per_gpu_step": n_cand,
        "replayed_positions_per_gpu_step": n_replay, "datagen_s": t_gen,
        "calls_gathered_per_step": sum(gathered) if gathered is not None else n_cand,
    }
    if rank == 0 and world == 1 and not args.no_e2e and L == L_SARS:
        res["end_to_end"] = end_to_end(args, 0)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline(args)
        res["cpu_baseline"]["cores_available"] = len(os.sched_getaffinity(0))
    if rank == 0:
        print(json.dumps(res))
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
