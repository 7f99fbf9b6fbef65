"""PileupEngine — Python front end of the MI355X engine context (include/spings_gpu.h).

One engine = one spg_ctx = one HIP device's accumulators for ``n_pos`` reference positions.
It replaces LiveVariantCaller's ``memory`` dict and the statistics loop
(variant_caller/live_variant_caller.py:37-231, utils.py:9-24).  Calls are serialised with a
lock: the C context is not re-entrant, while the reference drives its engine from daemon
threads (client_server/vc_queue.py:99-111).
"""
from __future__ import annotations

import ctypes as C
import math
import threading
import weakref
from typing import Dict, List, Optional

import numpy as np

from . import _native as N


def eps_lut() -> np.ndarray:
    """from_phred_scale (utils.py:9-10) with the same math.pow, so device eps are bit-identical."""
    return np.array([math.pow(10, q / -10) for q in range(256)], dtype=np.float64)


class PileupEngine:
    def __init__(self, n_pos: int, min_base_quality: int = 30, min_total_depth: int = 10,
                 min_allele_depth: int = 5, min_evidence_ratio: float = 0.10, device: int = 0,
                 reference: Optional[str] = None, calls_only: bool = False):
        """``calls_only`` (SPG_P_CALLS_ONLY): compute exactly what prepare_variants() emits; table GLs
        that only the engine's own per-position table would show may read NaN (SPG_F_PARTIAL)."""
        self._L = N.gpu_lib()
        self._lock = threading.RLock()
        self.n_pos = int(n_pos)
        self.device = int(device)
        self.calls_only = bool(calls_only)
        self.params = N.SpgParams(int(min_base_quality), int(min_total_depth), int(min_allele_depth),
                                  N.SPG_P_CALLS_ONLY if calls_only else 0, float(min_evidence_ratio))
        h = C.c_void_p()
        N.check(self._L.spg_create(self.device, self.n_pos, C.byref(self.params), C.byref(h)), "spg_create")
        self._h = h
        self._lut = eps_lut()
        N.check(self._L.spg_set_eps_lut(self._h, N.ptr(self._lut)), "spg_set_eps_lut")
        self._borrowed = []          # device tensors kept alive while borrowed as history
        self.reference = None
        if reference is not None:
            self.set_reference(reference)

    # -- lifecycle --------------------------------------------------------------------------
    def close(self):
        pool = getattr(self, "_stage_pool", None)
        if pool is not None:                           # (a staging reservation in flight finishes first)
            pool.shutdown(wait=True)
            self._stage_pool = self._stage_job = None
        with self._lock:
            self._ext = None
            if getattr(self, "_h", None):
                self._L.spg_destroy(self._h)
                self._h = None
            self._borrowed = []

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def reset(self):
        """reset_memory (live_variant_caller.py:37-38)."""
        with self._lock:
            N.check(self._L.spg_reset(self._h), "spg_reset")
            self._borrowed = []

    def set_reference(self, seq: str):
        """fastaFile.fetch (:78): REF chars for first visits."""
        with self._lock:
            b = seq.encode("latin-1") if isinstance(seq, str) else bytes(seq)
            N.check(self._L.spg_set_reference(self._h, b, len(b)), "spg_set_reference")
            self.reference = seq

    # -- hot path ---------------------------------------------------------------------------
    def accumulate(self, pos_begin: int, offsets, codes, quals, borrow: bool = False, n_entries=None,
                   trusted: bool = False):
        """process_pileup_column over one CSR batch (:74-103).  numpy arrays are host buffers;
        torch tensors on this engine's device are consumed in place (``borrow`` keeps them as
        replay history without a copy — they must stay alive until reset())."""
        with self._lock:
            if isinstance(offsets, np.ndarray) or isinstance(offsets, (list, tuple)):
                o = np.ascontiguousarray(offsets, dtype=np.uint64)
                c = np.ascontiguousarray(codes, dtype=np.uint8)
                q = np.ascontiguousarray(quals, dtype=np.uint8)
                n_cols = len(o) - 1
                if len(c) != len(q):
                    raise ValueError("codes and quals differ in length")
                # (trusted: the CSR comes from the pileup library, SPG_IN_TRUSTED skips the O(E) scan)
                N.check(self._L.spg_accumulate_ex(self._h, int(pos_begin), n_cols, N.ptr(o), N.ptr(c), N.ptr(q),
                                                  len(c), N.SPG_IN_TRUSTED if trusted else 0), "spg_accumulate")
            else:
                import torch
                for t in (offsets, codes, quals):
                    if not t.is_cuda or t.device.index != self.device or not t.is_contiguous():
                        raise ValueError("device inputs must be contiguous tensors on the engine's device")
                if offsets.dtype not in (torch.int64, torch.uint64) or codes.dtype != torch.uint8 or quals.dtype != torch.uint8:
                    raise ValueError("device inputs: offsets int64, codes/quals uint8")
                # order the engine's stream after the producer's work on torch's current stream
                # (a device-side wait, no host synchronisation)
                self._torch_stream().wait_stream(torch.cuda.current_stream(self.device))
                flags = N.SPG_IN_DEVICE | (N.SPG_IN_BORROW if borrow else 0)
                n_cols = offsets.numel() - 1
                if n_entries is None:
                    n_entries = int(offsets[-1].item())
                if borrow and (codes.numel() < n_entries + 16 or quals.numel() < n_entries + 16):
                    raise ValueError("borrowed device buffers need >= 16 bytes of padding past the last entry")
                N.check(self._L.spg_accumulate_ex(self._h, int(pos_begin), n_cols, N.ptr(offsets), N.ptr(codes),
                                                  N.ptr(quals), int(n_entries), flags), "spg_accumulate_ex")
                if borrow:
                    self._borrowed.append((offsets, codes, quals))

    def accumulate_batches(self, batches, device: bool = False, borrow: bool = False):
        """Many batches in one call (spg_accumulate_batches): ``batches`` is a sequence of
        (pos_begin, offsets, codes, quals[, n_entries]) — numpy host arrays, or (``device=True``) torch
        tensors on this engine's device (``borrow`` keeps them as history without a copy; the caller
        keeps them alive until reset()).  Same result as one accumulate() per batch, in order."""
        with self._lock:
            rec = np.zeros(len(batches), N.BATCH_DTYPE)
            keep = []
            for i, b in enumerate(batches):
                pb, off, c, q = b[:4]
                if device:
                    n = int(b[4]) if len(b) > 4 else int(off[-1].item())
                    rec[i] = (int(pb), off.numel() - 1, off.data_ptr(), c.data_ptr(), q.data_ptr(), n)
                else:
                    off = np.ascontiguousarray(off, dtype=np.uint64)
                    c = np.ascontiguousarray(c, dtype=np.uint8)
                    q = np.ascontiguousarray(q, dtype=np.uint8)
                    if len(c) != len(q):
                        raise ValueError("codes and quals differ in length")
                    rec[i] = (int(pb), len(off) - 1, off.ctypes.data, c.ctypes.data, q.ctypes.data, len(c))
                keep.append((off, c, q))
            flags = 0
            if device:
                import torch
                self._torch_stream().wait_stream(torch.cuda.current_stream(self.device))
                flags = N.SPG_IN_DEVICE | (N.SPG_IN_BORROW if borrow else 0)
            N.check(self._L.spg_accumulate_batches(self._h, N.ptr(rec), len(rec), flags), "spg_accumulate_batches")
            if device and borrow:
                self._borrowed.extend(keep)

    def accumulate_samples(self, pos_begin: int, offsets, first_sample, codes, quals, n_samples: int,
                           borrow: bool = False, n_entries=None):
        """spg_accumulate_samples: ``n_samples`` BAMs over one coordinate range as ONE column-major
        batch (column c = sample 0's entries at c, then sample 1's, ...; see ``samples_to_columns``),
        equal to one accumulate() per sample in order.  ``first_sample`` (u32 per column, or None)
        names the first sample with an entry at each column.  numpy host arrays or torch tensors on
        this engine's device (``borrow``: kept as history without a copy)."""
        with self._lock:
            if isinstance(offsets, np.ndarray):
                o = np.ascontiguousarray(offsets, dtype=np.uint64)
                c = np.ascontiguousarray(codes, dtype=np.uint8)
                q = np.ascontiguousarray(quals, dtype=np.uint8)
                fs = None if first_sample is None else np.ascontiguousarray(first_sample, dtype=np.uint32)
                N.check(self._L.spg_accumulate_samples(self._h, int(pos_begin), len(o) - 1, int(n_samples), N.ptr(o),
                                                       N.ptr(fs) if fs is not None else None, N.ptr(c), N.ptr(q),
                                                       len(c), 0), "spg_accumulate_samples")
            else:
                import torch
                self._torch_stream().wait_stream(torch.cuda.current_stream(self.device))
                n = int(offsets[-1].item()) if n_entries is None else int(n_entries)
                flags = N.SPG_IN_DEVICE | (N.SPG_IN_BORROW if borrow else 0)
                N.check(self._L.spg_accumulate_samples(self._h, int(pos_begin), offsets.numel() - 1, int(n_samples),
                                                       N.ptr(offsets),
                                                       N.ptr(first_sample) if first_sample is not None else None,
                                                       N.ptr(codes), N.ptr(quals), n, flags), "spg_accumulate_samples")
                if borrow:
                    self._borrowed.append((offsets, first_sample, codes, quals))

    def accumulate_records(self, rec: np.ndarray, device: bool = True, borrow: bool = True):
        """spg_accumulate_batches over prebuilt spg_batch records (N.BATCH_DTYPE), e.g.
        synth_device.DeviceBatches.records(): one binding call for thousands of batches.  The caller
        keeps the buffers alive (borrowed device inputs) until reset()."""
        rec = np.ascontiguousarray(rec, dtype=N.BATCH_DTYPE)
        with self._lock:
            flags = 0
            if device:
                import torch
                self._torch_stream().wait_stream(torch.cuda.current_stream(self.device))
                flags = N.SPG_IN_DEVICE | (N.SPG_IN_BORROW if borrow else 0)
            N.check(self._L.spg_accumulate_batches(self._h, N.ptr(rec), len(rec), flags), "spg_accumulate_batches")

    def accumulate_bam_records(self, batch):
        """process_bam's accumulate step from a records plan (pileup.AlignmentFile.pileup_records): the inflated
        BAM and per-read index go to HBM and the device-side pileup writes the batch (spg_accumulate_records).
        Pinned plan buffers are copied asynchronously: keep ``batch`` open until wait_ticket(input_ticket())
        taken after this call returns."""
        r = batch.records()
        with self._lock:
            N.check(self._L.spg_accumulate_records(self._h, C.byref(r), 0), "spg_accumulate_records")

    # -- a BAM kept in HBM (spg_bam_*) ------------------------------------------------------
    def bam_open(self, bmap, tid: int, params) -> Optional[int]:
        """spg_bam_open: the BAM's compressed bytes (pileup.BamMap) to HBM, inflated and scanned there; returns the
        number of reads of contig ``tid`` the stepper keeps, or None when the BAM is not handled on the device (a
        member the GPU could not inflate, record chains that disagree: plan it on the host instead)."""
        i = bmap.info
        flt = N.SpgBamFilter(N.SPP_STEPPER[params.stepper], int(params.flag_filter), int(params.min_mapping_quality), 0)
        n = C.c_int64()
        with self._lock:
            rc = self._L.spg_bam_open(self._h, i.comp, i.comp_bytes, i.members, i.n_members, i.body, int(tid), i.n_ref,
                                      C.byref(flt), C.byref(n))
            if rc == 1:
                self.bam_fallback = self._L.spg_last_error().decode(errors="replace")
                return None
            N.check(rc, "spg_bam_open")
        return n.value

    def bam_slot(self, slot: int):
        """spg_bam_slot: the device BAM slot (0 / 1) the next bam_* calls use (two BAMs open at once)."""
        with self._lock:
            N.check(self._L.spg_bam_slot(self._h, int(slot)), "spg_bam_slot")
            self._bam_slot = int(slot)

    def bam_upload(self, bmap, slot: int):
        """spg_bam_upload: start copying a BAM's compressed bytes (pileup.BamMap, kept open until its bam_open in that
        slot returns) into device slot ``slot``; that bam_open then waits for the copy instead of making its own."""
        i = bmap.info
        with self._lock:
            N.check(self._L.spg_bam_upload(self._h, int(slot), i.comp, i.comp_bytes, i.members, i.n_members),
                    "spg_bam_upload")

    def bam_reads(self, n: int) -> Dict[str, np.ndarray]:
        """spg_bam_reads_copy: the open BAM's kept reads' fixed fields (pinned host arrays per BAM slot, reused
        across that slot's BAMs)."""
        slot = getattr(self, "_bam_slot", 0)
        allb = getattr(self, "_bam_bufs", None)
        if allb is None:
            allb = self._bam_bufs = {}
        bufs = allb.get(slot)
        if bufs is None or len(bufs["pos"]) < n:
            cap = max(1024, int(n * 1.125))
            bufs = {name: pinned_empty(cap, dt) for name, dt in N.BAM_READ_FIELDS}
            allb[slot] = bufs
        out = {name: a[:n] for name, a in bufs.items()}
        r = N.SpgBamReads(*[out[name].ctypes.data for name, _ in N.BAM_READ_FIELDS])
        with self._lock:
            N.check(self._L.spg_bam_reads_copy(self._h, C.byref(r)), "spg_bam_reads_copy")
        return out

    def bam_accumulate(self, batch) -> bool:
        """spg_bam_accumulate: a device plan (pileup.AlignmentFile.pileup_fields) — mate-overlap tweak, then the CSR
        entries written from the BAM in HBM (k_pileup_fill) and accumulated.  False when the plan was refused (two
        paired reads whose names differ behind equal hashes: plan the BAM on the host).  Keep ``batch`` open until
        wait_ticket(input_ticket()) taken after this call."""
        v = batch.device_plan()
        with self._lock:
            rc = self._L.spg_bam_accumulate(self._h, C.byref(v), 0)
            if rc == 1:
                self.bam_fallback = self._L.spg_last_error().decode(errors="replace")
                return False
            N.check(rc, "spg_bam_accumulate")
        return True

    def bam_plan_build(self, max_depth: int, ignore_overlaps: bool = True):
        """spg_bam_plan_build: the open BAM's pileup plan built in HBM — htslib's depth cap and mate pairing on the GPU
        (what AlignmentFile.pileup_fields computes on the host from bam_reads).  The plan (device pointers, valid until
        this slot's next bam_open) for bam_accumulate_planned, or None when the device declined (bam_fallback says
        why: plan on the host)."""
        p = N.SpgBamPlan()
        with self._lock:
            rc = self._L.spg_bam_plan_build(self._h, int(max_depth), 1 if ignore_overlaps else 0, C.byref(p))
            if rc == 1:
                self.bam_fallback = self._L.spg_last_error().decode(errors="replace")
                return None
            N.check(rc, "spg_bam_plan_build")
        return p

    def bam_accumulate_planned(self, plan) -> bool:
        """spg_bam_accumulate of a bam_plan_build plan (SPG_IN_DEVICE).  False when refused (two paired reads whose
        names differ behind equal hashes: plan the BAM on the host)."""
        with self._lock:
            rc = self._L.spg_bam_accumulate(self._h, C.byref(plan), N.SPG_IN_DEVICE)
            if rc == 1:
                self.bam_fallback = self._L.spg_last_error().decode(errors="replace")
                return False
            N.check(rc, "spg_bam_accumulate")
        return True

    def bam_plan_arrays(self, plan) -> Dict[str, np.ndarray]:
        """A bam_plan_build plan's arrays on the host (spg_bam_plan_download; tests)."""
        nc, nk, npr = max(0, int(plan.n_cols)), int(plan.n_kept), int(plan.n_pairs)
        out = {"offsets": np.zeros(nc + 1, np.uint64), "kept": np.zeros(nk, np.uint32), "pair_a": np.zeros(npr, np.uint32),
               "pair_b": np.zeros(npr, np.uint32), "pair_col": np.zeros(npr, np.int64),
               "pair_orig": np.zeros(npr, np.uint64)}
        with self._lock:
            N.check(self._L.spg_bam_plan_download(self._h, C.byref(plan), *[N.ptr(out[k]) for k in
                                                                            ("offsets", "kept", "pair_a", "pair_b",
                                                                             "pair_col", "pair_orig")]),
                    "spg_bam_plan_download")
        return out

    def bam_inflate_ms(self) -> float:
        ms = C.c_float()
        N.check(self._L.spg_bam_inflate_ms(self._h, C.byref(ms)), "spg_bam_inflate_ms")
        return ms.value

    def bam_inflate_fallbacks(self) -> int:
        """members of the last BAM opened in HBM that the parallel inflater left to the one-lane-per-member decoder"""
        n = C.c_int64()
        N.check(self._L.spg_bam_inflate_fallbacks(self._h, C.byref(n)), "spg_bam_inflate_fallbacks")
        return n.value

    def bam_release(self):
        """Free the BAM buffers in HBM (spg_bam_release)."""
        with self._lock:
            N.check(self._L.spg_bam_release(self._h), "spg_bam_release")

    def wait_input(self):
        """Block until every input copy enqueued so far has landed (pinned host buffers are free)."""
        with self._lock:
            N.check(self._L.spg_wait_input(self._h), "spg_wait_input")

    def set_history_cap(self, nbytes: int):
        """Bound the HBM the engine's own batch copies (the replay history) may hold: past it, the oldest
        folded batches move to pinned host memory (spg_set_history_cap; 0 = no cap)."""
        with self._lock:
            N.check(self._L.spg_set_history_cap(self._h, int(nbytes)), "spg_set_history_cap")

    def history_resident(self):
        """(owned history bytes in HBM, batches spilled to host, arena bytes allocated)."""
        a, b, d = C.c_int64(), C.c_int64(), C.c_int64()
        with self._lock:
            N.check(self._L.spg_history_resident(self._h, C.byref(a), C.byref(b), C.byref(d)), "spg_history_resident")
        return a.value, b.value, d.value

    PATHS = ("record_runs", "materializations", "full_finalizes", "sparse_finalizes", "counted_finalizes",
             "fused_deep_finalizes", "fused_shallow_finalizes", "batches_counted", "mid_counted_finalizes")

    def path_counters(self) -> Dict[str, int]:
        """Which engine paths ran since creation (spg_path_counters)."""
        a = (C.c_int64 * len(self.PATHS))()
        with self._lock:
            N.check(self._L.spg_path_counters(self._h, a, len(self.PATHS)), "spg_path_counters")
        return dict(zip(self.PATHS, list(a)))

    def input_ticket(self) -> int:
        """Ticket of the latest host-input batch copy enqueued (spg_input_ticket)."""
        t = C.c_uint64()
        with self._lock:
            N.check(self._L.spg_input_ticket(self._h, C.byref(t)), "spg_input_ticket")
        return t.value

    def wait_ticket(self, ticket: int):
        """Block until host-input copy #ticket has landed, not the ones enqueued after it."""
        with self._lock:
            N.check(self._L.spg_wait_ticket(self._h, int(ticket)), "spg_wait_ticket")

    def _torch_stream(self):
        if getattr(self, "_ext", None) is None:
            import torch
            st = C.c_void_p()
            N.check(self._L.spg_stream(self._h, C.byref(st)), "spg_stream")
            self._ext = torch.cuda.ExternalStream(st.value, device=torch.device("cuda", self.device))
        return self._ext

    def finalize(self):
        """prepare_variants (:120-231): per-position table + candidates, on device."""
        with self._lock:
            N.check(self._L.spg_finalize(self._h), "spg_finalize")

    def sync(self):
        with self._lock:
            N.check(self._L.spg_sync(self._h), "spg_sync")

    def copy_candidates_device(self, dst, cap=None):
        """Call table -> a torch uint8 device tensor (u64 count, then spg_candidate records)."""
        cap = (dst.numel() - 8) // N.CANDIDATE_DTYPE.itemsize if cap is None else cap
        import torch
        with self._lock:
            N.check(self._L.spg_copy_candidates_device(self._h, N.ptr(dst), int(cap)), "spg_copy_candidates_device")
            # consumers on torch's current stream (e.g. a torch.distributed gather) wait on the copy
            torch.cuda.current_stream(self.device).wait_stream(self._torch_stream())

    def last_kernel_ms(self):
        a, f = C.c_float(), C.c_float()
        with self._lock:
            N.check(self._L.spg_last_kernel_ms(self._h, C.byref(a), C.byref(f)), "spg_last_kernel_ms")
        return a.value, f.value

    def set_timing(self, level: int):
        """Timing events recorded from now on: 2 accumulate + finalize, 1 accumulate only, 0 none."""
        with self._lock:
            N.check(self._L.spg_set_timing(self._h, int(level)), "spg_set_timing")

    def kernel_times(self, cap: int = 64):
        """(accumulate_ms, finalize_ms) arrays of every step finalized since the previous call."""
        a = np.zeros(cap, np.float32)
        f = np.zeros(cap, np.float32)
        n = C.c_int64()
        with self._lock:
            N.check(self._L.spg_kernel_times(self._h, N.ptr(a), N.ptr(f), int(cap), C.byref(n)), "spg_kernel_times")
        return a[:n.value].astype(np.float64), f[:n.value].astype(np.float64)

    def position_entries(self, pos: int, upto: Optional[int] = None):
        """(codes, quals) of every entry at ``pos`` over the history (its first ``upto`` batches), in accumulate order
        (spg_position_entries_upto)."""
        n = C.c_int64()
        ub = (1 << 62) if upto is None else int(upto)
        with self._lock:
            N.check(self._L.spg_position_entries_upto(self._h, int(pos), ub, None, None, 0, C.byref(n)),
                    "spg_position_entries")
            codes = np.zeros(n.value, np.uint8)
            quals = np.zeros(n.value, np.uint8)
            if n.value:
                N.check(self._L.spg_position_entries_upto(self._h, int(pos), ub, N.ptr(codes), N.ptr(quals), n.value,
                                                          C.byref(n)), "spg_position_entries")
        return codes, quals

    def history_count(self) -> int:
        """Batches accumulated since reset() (spg_history_count)."""
        n = C.c_int64()
        with self._lock:
            N.check(self._L.spg_history_count(self._h, C.byref(n)), "spg_history_count")
        return n.value

    def history(self, start: int = 0, min_bq: Optional[int] = None):
        """The accumulated batches since reset() from batch `start` on, as host copies:
        [(pos_begin, offsets, codes, quals)] (min_bq: compacted as the checkpoint keeps them, iter_history)."""
        return list(self.iter_history(start, min_bq))

    def iter_history(self, start: int = 0, min_bq: Optional[int] = None, staged: bool = False):
        """The batches one at a time (a long history never sits on the host at once).  min_bq: each batch as
        create_checkpoint keeps it — the entries with q >= min_bq plus a first-entry marker per column whose entries all
        fail (spg_history_copy_compact: compacted in HBM, only the kept bytes cross PCIe).  staged: the arrays are views
        of the engine's pinned staging (DMA'd, no bounce copy), valid until the next batch is yielded."""
        n = self.history_count()
        for i in range(max(0, int(start)), n):
            with self._lock:
                pb, nc, ne = C.c_int64(), C.c_int64(), C.c_uint64()
                N.check(self._L.spg_history_info(self._h, i, C.byref(pb), C.byref(nc), C.byref(ne)),
                        "spg_history_info")
                if staged:
                    off, codes, quals = self._staging(nc.value + 1, ne.value)
                else:
                    off = np.zeros(nc.value + 1, np.uint64)
                    codes = np.empty(ne.value, np.uint8)
                    quals = np.empty(ne.value, np.uint8)
                if min_bq is None:
                    N.check(self._L.spg_history_copy(self._h, i, N.ptr(off), N.ptr(codes), N.ptr(quals)),
                            "spg_history_copy")
                else:
                    k = C.c_uint64()
                    N.check(self._L.spg_history_copy_compact(self._h, i, int(min_bq), N.ptr(off), N.ptr(codes),
                                                             N.ptr(quals), C.byref(k)), "spg_history_copy_compact")
                    codes, quals = codes[:k.value], quals[:k.value]   # (pages past k never touched)
            yield pb.value, off, codes, quals

    def iter_history_packed(self, start: int, min_bq: int, exc_cap: int = 1 << 20):
        """The batches as create_checkpoint writes them, packed (spg_history_copy_packed): per batch a dict of the
        compact CSR offsets, one byte per kept entry and the exception list (index, code, quality) of the entries the
        byte cannot hold — or, when the exceptions exceed exc_cap, the unpacked codes / quals.  Arrays are views of
        pinned staging, valid until the next batch is yielded."""
        n = self.history_count()
        for i in range(max(0, int(start)), n):
            with self._lock:
                pb, nc, ne = C.c_int64(), C.c_int64(), C.c_uint64()
                N.check(self._L.spg_history_info(self._h, i, C.byref(pb), C.byref(nc), C.byref(ne)), "spg_history_info")
                off, packed, _ = self._staging(nc.value + 1, ne.value, two=False)
                xs = getattr(self, "_xstage", None)
                if xs is None or len(xs[1]) < exc_cap:
                    xs = (pinned_empty(exc_cap, np.uint64), pinned_empty(exc_cap), pinned_empty(exc_cap))
                    self._xstage = xs
                k, nx = C.c_uint64(), C.c_int64()
                N.check(self._L.spg_history_copy_packed(self._h, i, int(min_bq), N.ptr(off), N.ptr(packed), C.byref(k),
                                                        N.ptr(xs[0]), N.ptr(xs[1]), N.ptr(xs[2]), int(exc_cap),
                                                        C.byref(nx)), "spg_history_copy_packed")
                if nx.value <= exc_cap:
                    m = nx.value
                    ent = {"pos": pb.value, "off": off, "packed": packed[:k.value], "xi": xs[0][:m], "xc": xs[1][:m],
                           "xq": xs[2][:m]}
                else:
                    off, codes, quals = self._staging(nc.value + 1, ne.value)
                    N.check(self._L.spg_history_copy_compact(self._h, i, int(min_bq), N.ptr(off), N.ptr(codes),
                                                             N.ptr(quals), C.byref(k)), "spg_history_copy_compact")
                    ent = {"pos": pb.value, "off": off, "codes": codes[:k.value], "quals": quals[:k.value]}
            yield ent

    CK_EXC_CAP = 1 << 22

    def copy_history_packed(self, start: int, min_bq: int, exc_cap: int = CK_EXC_CAP):
        """The batches [start, history_count()) packed as iter_history_packed yields them, all copied at once into
        pinned buffers of their own (reused by the next call: a write-behind checkpoint holds them until its file is
        written).  None when the batches' exceptions exceed exc_cap (the caller then streams iter_history_packed)."""
        n = self.history_count()
        infos = []
        with self._lock:
            for i in range(max(0, int(start)), n):
                pb, nc, ne = C.c_int64(), C.c_int64(), C.c_uint64()
                N.check(self._L.spg_history_info(self._h, i, C.byref(pb), C.byref(nc), C.byref(ne)), "spg_history_info")
                infos.append((i, pb.value, nc.value, ne.value))
            n_off = sum(nc + 1 for _, _, nc, _ in infos)
            n_ent = sum(ne for _, _, _, ne in infos)
            self._take_reservation()
            st = getattr(self, "_ckstage", None)
            if st is None or len(st[0]) < n_off or len(st[1]) < n_ent or len(st[2]) < exc_cap:
                st = (pinned_empty(max(n_off, int(n_off * 1.125)), np.uint64), pinned_empty(max(16, int(n_ent * 1.125))),
                      pinned_empty(exc_cap, np.uint64), pinned_empty(exc_cap), pinned_empty(exc_cap))
                self._ckstage = st
            out, o0, e0, x0 = [], 0, 0, 0
            for i, pb, nc, ne in infos:
                off, packed = st[0][o0:o0 + nc + 1], st[1][e0:e0 + ne]
                xi, xc, xq = st[2][x0:], st[3][x0:], st[4][x0:]
                k, nx = C.c_uint64(), C.c_int64()
                N.check(self._L.spg_history_copy_packed(self._h, i, int(min_bq), N.ptr(off), N.ptr(packed), C.byref(k),
                                                        N.ptr(xi), N.ptr(xc), N.ptr(xq), int(len(xi)), C.byref(nx)),
                        "spg_history_copy_packed")
                if nx.value > len(xi):
                    return None
                m = nx.value
                out.append({"pos": pb, "off": off, "packed": packed[:k.value], "xi": xi[:m], "xc": xc[:m], "xq": xq[:m]})
                o0, e0, x0 = o0 + nc + 1, e0 + ne, x0 + m
        return out

    def _staging(self, n_off: int, n_entries: int, two: bool = True):
        """Pinned host views (offsets, codes, quals) for history copies, grown as needed and reused (the quals array
        only when `two`: a packed checkpoint needs one byte per entry; else None).  A reservation made ahead of time
        (reserve_staging) is taken over here."""
        self._take_reservation()
        st = getattr(self, "_stage", None)
        if st is None or len(st[0]) < n_off or len(st[1]) < n_entries:
            st = [pinned_empty(max(n_off, int(n_off * 1.125)), np.uint64), pinned_empty(max(16, int(n_entries * 1.125))),
                  None]
            self._stage = st
        if two and (st[2] is None or len(st[2]) < n_entries):
            st[2] = pinned_empty(max(16, len(st[1])))
        return st[0][:n_off], st[1][:n_entries], (st[2][:n_entries] if two else None)

    def _take_reservation(self):
        """Install the staging reserve_staging allocated (waits for it) where it is larger than the current one."""
        job = getattr(self, "_stage_job", None)
        if job is None:
            return
        self._stage_job = None
        got = job.result()
        if got is None:
            return
        name, arrs = got
        cur = getattr(self, name, None)
        if cur is None or len(arrs[1]) > len(cur[1]) or len(arrs[0]) > len(cur[0]):
            setattr(self, name, arrs)

    def reserve_staging(self, n_off: int, n_entries, write_behind: bool = False):
        """Allocate the checkpoint's pinned staging (iter_history_packed: offsets + one byte per entry) for a batch of
        about this size on a helper thread, while the caller goes on (pinning ~0.4 GB of pages takes tens of ms: the
        first create_checkpoint of a caller used to pay it).  `n_entries`: a number, or a callable the helper evaluates
        (an estimate from arrays the caller keeps unchanged meanwhile).  No-op when the staging already holds that size;
        a short estimate only means the checkpoint grows the staging itself, as before.  `write_behind`: the staging of
        copy_history_packed (a write-behind checkpoint) instead of iter_history_packed's."""
        if getattr(self, "_stage_job", None) is not None:
            return
        if getattr(self, "_stage_pool", None) is None:
            from concurrent.futures import ThreadPoolExecutor
            self._stage_pool = ThreadPoolExecutor(1, thread_name_prefix="spg-stage")
        name = "_ckstage" if write_behind else "_stage"
        st = getattr(self, name, None)
        have = (len(st[0]), len(st[1])) if st is not None else (0, 0)

        def alloc():
            ne = int(n_entries() if callable(n_entries) else n_entries)
            if have[0] >= n_off and have[1] >= ne:
                return None
            arrs = [pinned_empty(max(n_off, int(n_off * 1.125)), np.uint64), pinned_empty(max(16, int(ne * 1.125)))]
            if write_behind:
                xc = self.CK_EXC_CAP
                arrs += [pinned_empty(xc, np.uint64), pinned_empty(xc), pinned_empty(xc)]
            else:
                arrs.append(None)
            return name, arrs
        self._stage_job = self._stage_pool.submit(alloc)

    # -- results ------------------------------------------------------------------------------
    def table(self, pos0: int = 0, n: Optional[int] = None) -> Dict[str, np.ndarray]:
        n = self.n_pos - pos0 if n is None else n
        out = dict(depth=np.zeros(n, np.uint32), counts=np.zeros((n, N.SPG_NCOUNT), np.uint32),
                   gl=np.zeros((n, N.SPG_NSLOT), np.float64), flags=np.zeros(n, np.uint8),
                   order=np.zeros(n, np.uint32), first_batch=np.zeros(n, np.uint32))
        with self._lock:
            N.check(self._L.spg_get_table(self._h, pos0, n, *[N.ptr(out[k]) for k in
                                                              ("depth", "counts", "gl", "flags", "order",
                                                               "first_batch")]), "spg_get_table")
        return out

    def counts(self):
        nc, nd = C.c_int64(), C.c_int64()
        with self._lock:
            N.check(self._L.spg_count(self._h, C.byref(nc), C.byref(nd)), "spg_count")
        return nc.value, nd.value

    def candidates(self) -> np.ndarray:
        """Variants ordered like prepare_variants(): memory insertion order (first batch, then
        position — htslib emits columns in coordinate order), then snvs dict order."""
        with self._lock:
            nc, _ = self.counts()
            arr = np.zeros(nc, N.CANDIDATE_DTYPE)
            got = C.c_int64()
            N.check(self._L.spg_get_candidates(self._h, N.ptr(arr), nc, C.byref(got)), "spg_get_candidates")
        arr = arr[:got.value]
        return arr[np.lexsort((arr["rank"], arr["pos"], arr["first_batch"]))]

    def details(self) -> np.ndarray:
        with self._lock:
            _, nd = self.counts()
            arr = np.zeros(nd, N.DETAIL_DTYPE)
            got = C.c_int64()
            N.check(self._L.spg_get_details(self._h, N.ptr(arr), nd, C.byref(got)), "spg_get_details")
        return arr[:got.value]

    # -- reference-shaped views -----------------------------------------------------------------
    def variants(self) -> List[dict]:
        """The list prepare_variants() returns (live_variant_caller.py:170-185)."""
        return self._variants_of(self.candidates())

    @staticmethod
    def _variants_of(cands) -> List[dict]:
        out = []
        for r in cands:
            gl = 0 if r["gl_zero"] else float(r["gl"])
            out.append({
                "start": int(r["pos"]), "stop": int(r["pos"]) + 1,
                "alleles": (chr(r["ref"]), chr(r["alt"])),
                "qual": np.float64(r["qual"]),
                "info": {"DP": int(r["dp"]), "AD": int(r["ad"]), "GL": gl, "PL": int(r["pl"]),
                         "SCORE": int(r["score"])},
            })
        return out

    def memory_summary(self):
        """[pos, REF, totalDepth, [[allele, count] in snvs dict order]] in memory insertion order."""
        t = self.table()
        det = {int(d["pos"]): d for d in self.details()}
        present = np.nonzero(t["flags"] & N.SPG_F_PRESENT)[0]
        order = present[np.lexsort((present, t["first_batch"][present]))]
        ref = self.reference
        out = []
        for p in order.tolist():
            if p in det:
                d = det[p]
                alle = [[N.NIBBLE[d["code"][k]], int(d["count"][k])] for k in range(d["n_alleles"])]
            else:
                o = int(t["order"][p])
                alle = [[N.SLOT_CHARS[(o >> (3 + 3 * i)) & 7], int(t["counts"][p][(o >> (3 + 3 * i)) & 7])]
                        for i in range(o & 7)]
            out.append([p, ref[p] if ref is not None else None, int(t["depth"][p]), alle])
        return out

    def gl_table(self):
        """{pos: {allele: GL}} for evaluated positions, alleles in dict order."""
        t = self.table()
        det = {int(d["pos"]): d for d in self.details()}
        out = {}
        for p in np.nonzero(t["flags"] & N.SPG_F_EVALUATED)[0].tolist():
            if p in det:
                d = det[p]
                out[p] = {N.NIBBLE[d["code"][k]]: float(d["gl"][k]) for k in range(d["n_alleles"])}
            else:
                o = int(t["order"][p])
                out[p] = {N.SLOT_CHARS[(o >> (3 + 3 * i)) & 7]: float(t["gl"][p][(o >> (3 + 3 * i)) & 7])
                          for i in range(o & 7)}
        return out


def samples_to_columns(batches):
    """Per-sample CSR batches over one range [(pos_begin, offsets, codes, quals)] -> the column-major
    multi-sample batch of spg_accumulate_samples: (pos_begin, offsets, first_sample, codes, quals)."""
    pbs = {int(b[0]) for b in batches}
    ncs = {len(b[1]) - 1 for b in batches}
    if len(pbs) != 1 or len(ncs) != 1:
        raise ValueError("samples_to_columns: every sample batch must cover the same columns")
    pb, C, S = pbs.pop(), ncs.pop(), len(batches)
    lens = np.stack([np.diff(np.asarray(b[1], np.int64)) for b in batches])      # [S, C]
    tot = lens.sum(axis=0)
    off = np.zeros(C + 1, np.uint64)
    np.cumsum(tot, out=off[1:])
    # destination of sample s's column c: off[c] + lens[:s, c].sum()
    start = off[:-1].astype(np.int64)[None, :] + np.cumsum(lens, axis=0) - lens
    E = int(off[-1])
    codes = np.empty(E, np.uint8)
    quals = np.empty(E, np.uint8)
    for s, b in enumerate(batches):
        src_off = np.asarray(b[1], np.int64)
        col = np.repeat(np.arange(C), lens[s])
        dst = start[s][col] + (np.arange(len(col)) - src_off[:-1][col])
        codes[dst] = b[2]
        quals[dst] = b[3]
    has = lens > 0
    first = np.where(has.any(axis=0), has.argmax(axis=0), 0).astype(np.uint32)
    return pb, off, first, codes, quals


def pinned_empty(n: int, dtype=np.uint8) -> np.ndarray:
    """A numpy array in pinned (page-locked) host memory (spg_host_alloc): CSR inputs staged here are
    copied to HBM asynchronously (engine.wait_input() before reusing the buffer)."""
    dtype = np.dtype(dtype)
    nbytes = max(1, int(n) * dtype.itemsize)
    L = N.gpu_lib()
    p = C.c_void_p()
    N.check(L.spg_host_alloc(nbytes, C.byref(p)), "spg_host_alloc")
    buf = (C.c_uint8 * nbytes).from_address(p.value)
    weakref.finalize(buf, L.spg_host_free, C.c_void_p(p.value))
    return np.frombuffer(buf, dtype=dtype, count=int(n))


def device_count() -> int:
    n = C.c_int()
    N.check(N.gpu_lib().spg_device_count(C.byref(n)), "spg_device_count")
    return n.value
