"""Pileup front end: BAM/SAM contig -> CSR batch for the GPU engine.

Replaces ``pysam.AlignmentFile(path).pileup(min_mapping_quality=..., min_base_quality=...,
reference=contig)`` as called by ``LiveVariantCaller.process_bam``
(variant_caller/live_variant_caller.py:55-60).  The reading, read filtering, htslib depth cap
and CIGAR walk run in the host C++ library (include/spings_pileup.h); the base-quality filter
is applied by the GPU engine.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import List, Tuple

import numpy as np

from . import _native as N


def cpu_share() -> int:
    """CPUs this process may actually use: its affinity mask, capped by the cgroup CPU quota (cpu.max) when one is
    set — the GPU box's 16-CPU quota behind a 256-CPU affinity mask (profiles/r04s: 32 threads on it ran the
    records plan 10-15 % slower than 16 would)."""
    import os
    n = len(os.sched_getaffinity(0))
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, -(-int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return n


@dataclass
class PileupParams:
    """pysam pileup() keyword defaults (stepper 'all', max_depth 8000, ignore_overlaps True)."""
    stepper: str = "all"
    min_mapping_quality: int = 0
    max_depth: int = 8000
    ignore_overlaps: bool = True
    flag_filter: int = 0x704
    n_threads: int = 8
    inflate_device: int = -1          # records plans: BGZF members inflated on this GPU (-1: on the host's threads) ...
    inflate_min_members: int = 0      # ... for BAMs of at least this many members (0: 4096)

    def native(self) -> N.SppParams:
        p = N.SppParams()
        N.pileup_lib().spp_default_params(C.byref(p))
        p.stepper = N.SPP_STEPPER[self.stepper]
        p.min_mapping_quality = int(self.min_mapping_quality)
        p.max_depth = int(self.max_depth)
        p.ignore_overlaps = 1 if self.ignore_overlaps else 0
        p.flag_filter = int(self.flag_filter)
        p.n_threads = int(self.n_threads)
        p.inflate_device = int(self.inflate_device)
        p.inflate_min_members = int(self.inflate_min_members)
        if p.inflate_device >= 0:
            N.register_gpu_inflater()
        return p


class PileupBatch:
    """CSR batch owned by the native library: ``offsets`` u64[n_cols+1], ``codes``/``quals`` u8[E]
    (16 padding bytes follow both arrays), columns [pos_begin, pos_begin + n_cols)."""

    def __init__(self, handle, planned=False, records=False, device=False):
        L = N.pileup_lib()
        self.is_records = bool(records)
        self.is_device = bool(device)
        self._h = C.c_void_p(handle)
        pb, nc, ne, nu, nd = C.c_int64(), C.c_int64(), C.c_uint64(), C.c_int64(), C.c_int64()
        N.pcheck(L.spp_batch_info(self._h, C.byref(pb), C.byref(nc), C.byref(ne), C.byref(nu), C.byref(nd)),
                 "spp_batch_info")
        self.pos_begin, self.n_cols, self.n_entries = pb.value, nc.value, ne.value
        self.n_reads_used, self.n_reads_dropped = nu.value, nd.value
        if not planned:
            self._arrays()

    def fill(self, codes_buf=None, quals_buf=None):
        """Second phase of AlignmentFile.pileup_plan: write base codes / qualities into the given uint8
        arrays (>= n_entries + 16 each, e.g. pinned host memory reused across BAMs) or into the
        library's own allocation.  Returns self."""
        L = N.pileup_lib()
        if (codes_buf is None) != (quals_buf is None):
            raise ValueError("fill: give both buffers or neither")
        if codes_buf is not None:
            need = self.n_entries + 16
            if codes_buf.nbytes < need or quals_buf.nbytes < need:
                raise ValueError(f"fill: buffers must hold n_entries + 16 = {need} bytes")
            N.pcheck(L.spp_batch_fill(self._h, N.ptr(codes_buf), N.ptr(quals_buf)), "spp_batch_fill")
        else:
            N.pcheck(L.spp_batch_fill(self._h, None, None), "spp_batch_fill")
        self._arrays()
        return self

    def records(self) -> N.SpgRecords:
        """The records plan's spg_records view (valid until close())."""
        if not self.is_records:
            raise ValueError("records(): not a records plan (AlignmentFile.pileup_records)")
        r = N.SpgRecords()
        N.pcheck(N.pileup_lib().spp_batch_records(self._h, C.byref(r)), "spp_batch_records")
        return r

    def device_plan(self) -> N.SpgBamPlan:
        """A device plan's spg_bam_plan view (AlignmentFile.pileup_fields; valid until close())."""
        if not self.is_device:
            raise ValueError("device_plan(): not a device plan (AlignmentFile.pileup_fields)")
        v = N.SpgBamPlan()
        N.pcheck(N.pileup_lib().spp_batch_device_plan(self._h, C.byref(v)), "spp_batch_device_plan")
        return v

    def _arrays(self):
        L = N.pileup_lib()
        po, pc, pq = C.c_void_p(), C.c_void_p(), C.c_void_p()
        N.pcheck(L.spp_batch_arrays(self._h, C.byref(po), C.byref(pc), C.byref(pq)), "spp_batch_arrays")
        E = self.n_entries
        self.offsets = np.ctypeslib.as_array(C.cast(po, C.POINTER(C.c_uint64)), (self.n_cols + 1,))
        self.codes_padded = np.ctypeslib.as_array(C.cast(pc, C.POINTER(C.c_uint8)), (E + 16,))
        self.quals_padded = np.ctypeslib.as_array(C.cast(pq, C.POINTER(C.c_uint8)), (E + 16,))
        self.codes = self.codes_padded[:E]
        self.quals = self.quals_padded[:E]

    def close(self):
        if self._h:
            N.pileup_lib().spp_batch_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def arrays(self) -> Tuple[int, np.ndarray, np.ndarray, np.ndarray]:
        return self.pos_begin, self.offsets, self.codes, self.quals


class AlignmentFile:
    """Minimal pysam.AlignmentFile stand-in for the hot path: header targets + contig pileup."""

    def __init__(self, path: str, mode: str = "rb"):
        L = N.pileup_lib()
        h = C.c_void_p()
        N.pcheck(L.spp_open(str(path).encode(), C.byref(h)), f"open {path}")
        self._h = h
        n = C.c_int32()
        N.pcheck(L.spp_n_targets(h, C.byref(n)))
        self.references: List[str] = []
        self.lengths: List[int] = []
        for t in range(n.value):
            nm, ln = C.c_char_p(), C.c_int64()
            N.pcheck(L.spp_target(h, t, C.byref(nm), C.byref(ln)))
            self.references.append(nm.value.decode())
            self.lengths.append(ln.value)

    def get_reference_length(self, reference: str) -> int:
        return self.lengths[self.references.index(reference)]

    def pileup_batch(self, reference: str, params: PileupParams | None = None, start: int | None = None,
                     stop: int | None = None) -> PileupBatch:
        """The contig's pileup as one CSR batch; with start/stop only the columns [start, stop) (a
        coordinate shard: spp_pileup_region, identical to slicing the whole-contig batch)."""
        L = N.pileup_lib()
        tid = C.c_int32()
        N.pcheck(L.spp_target_id(self._h, reference.encode(), C.byref(tid)), "pileup")
        b = C.c_void_p()
        prm = (params or PileupParams()).native()
        if start is None and stop is None:
            N.pcheck(L.spp_pileup(self._h, tid.value, C.byref(prm), C.byref(b)), "pileup")
        else:
            lo = -(1 << 62) if start is None else int(start)
            hi = (1 << 62) if stop is None else int(stop)
            N.pcheck(L.spp_pileup_region(self._h, tid.value, lo, hi, C.byref(prm), C.byref(b)), "pileup")
        return PileupBatch(b.value)

    def pileup_plan(self, reference: str, params: PileupParams | None = None, start: int | None = None,
                    stop: int | None = None) -> PileupBatch:
        """First phase of the two-phase pileup (spp_pileup_plan): reads parsed, depth cap applied, CSR
        offsets and n_entries known; PileupBatch.fill() writes the entries (into caller buffers)."""
        L = N.pileup_lib()
        tid = C.c_int32()
        N.pcheck(L.spp_target_id(self._h, reference.encode(), C.byref(tid)), "pileup")
        b = C.c_void_p()
        prm = (params or PileupParams()).native()
        lo = -(1 << 63) if start is None else int(start)
        hi = (1 << 63) - 1 if stop is None else int(stop)
        N.pcheck(L.spp_pileup_plan(self._h, tid.value, lo, hi, C.byref(prm), C.byref(b)), "pileup")
        return PileupBatch(b.value, planned=True)

    def pileup_records(self, reference: str, params: PileupParams | None = None, start: int | None = None,
                       stop: int | None = None) -> PileupBatch:
        """Device-decode form of pileup_plan (spp_pileup_plan_records, BAM only): reads parsed, depth cap /
        overlap tweak applied, CSR offsets known; the entries are written on the GPU from the raw records
        (PileupEngine.accumulate_bam_records -> spg_accumulate_records)."""
        L = N.pileup_lib()
        tid = C.c_int32()
        N.pcheck(L.spp_target_id(self._h, reference.encode(), C.byref(tid)), "pileup")
        b = C.c_void_p()
        prm = (params or PileupParams()).native()
        lo = -(1 << 63) if start is None else int(start)
        hi = (1 << 63) - 1 if stop is None else int(stop)
        N.pcheck(L.spp_pileup_plan_records(self._h, tid.value, lo, hi, C.byref(prm), C.byref(b)), "pileup")
        return PileupBatch(b.value, planned=True, records=True)

    def tid(self, reference: str) -> int:
        t = C.c_int32()
        N.pcheck(N.pileup_lib().spp_target_id(self._h, reference.encode(), C.byref(t)), "pileup")
        return t.value

    def bam_map(self, n_threads: int = 8) -> "BamMap":
        """The BAM's compressed bytes (pinned under the allocator hook) and BGZF member table for spg_bam_open."""
        return BamMap(self, n_threads)

    def pileup_fields(self, reference: str, reads: dict, params: PileupParams | None = None) -> PileupBatch:
        """The device plan (spp_pileup_plan_fields): htslib's depth cap and mate pairing replayed on the reads' fixed
        fields (PileupEngine.bam_reads), the CSR offsets and the overlapping mate pairs — for
        PileupEngine.bam_accumulate, which writes the entries from the BAM in HBM."""
        f = N.SppReadFields()
        f.n = int(len(reads["pos"]))
        for name, dt in N.BAM_READ_FIELDS:
            a = reads[name]
            assert a.dtype == dt and a.flags.c_contiguous and len(a) >= f.n
            setattr(f, name, a.ctypes.data)
        prm = (params or PileupParams()).native()
        b = C.c_void_p()
        N.pcheck(N.pileup_lib().spp_pileup_plan_fields(self._h, self.tid(reference), C.byref(f), C.byref(prm), C.byref(b)),
                 "pileup")
        return PileupBatch(b.value, planned=True, device=True)

    def close(self):
        if self._h:
            N.pileup_lib().spp_close(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class BamMap:
    """spp_bam_map_open: a BAM's bytes in one host buffer + its BGZF members and header end (spg_bam_open's input)."""

    def __init__(self, f: AlignmentFile, n_threads: int = 8):
        self.info = N.SppBamMapInfo()
        h = C.c_void_p()
        N.pcheck(N.pileup_lib().spp_bam_map_open(f._h, int(n_threads), C.byref(h), C.byref(self.info)), "spp_bam_map_open")
        self._h = h

    def close(self):
        if self._h:
            N.pileup_lib().spp_bam_map_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def simulate_bam(path: str, contig: str, reference: str, depth: float, seed: int = 2, n_threads: int = 8,
                 **kw) -> int:
    """Write a synthetic coordinate-sorted BAM (include/spings_pileup.h spp_simulate_bam; SURVEY §8 d
    read model).  Extra keywords override spp_sim_params fields.  Returns the number of reads."""
    L = N.pileup_lib()
    p = N.SimParams()
    L.spp_default_sim_params(C.byref(p))
    p.depth, p.seed, p.n_threads = float(depth), int(seed), int(n_threads)
    for k, v in kw.items():
        setattr(p, k, v)
    n = C.c_int64()
    ref = reference.encode()
    N.pcheck(L.spp_simulate_bam(str(path).encode(), contig.encode(), ref, len(ref), C.byref(p), C.byref(n)),
             "spp_simulate_bam")
    return n.value


def synth_batch(reference: str, depth: float, lo: int = 0, hi: int | None = None, seed: int = 2, n_threads: int = 16,
                max_depth: int = 0, **kw) -> PileupBatch:
    """Synthetic CSR pileup of columns [lo, hi) generated natively (spp_synth_batch): the read model
    of SURVEY §8 d at column level, for configs too large for numpy (100,000x, chr1 30x)."""
    L = N.pileup_lib()
    p = N.SimParams()
    L.spp_default_sim_params(C.byref(p))
    p.depth, p.seed, p.n_threads = float(depth), int(seed), int(n_threads)
    for k, v in kw.items():
        setattr(p, k, v)
    ref = reference.encode()
    hi = len(ref) if hi is None else hi
    b = C.c_void_p()
    N.pcheck(L.spp_synth_batch(ref, len(ref), int(lo), int(hi), C.byref(p), int(max_depth), C.byref(b)),
             "spp_synth_batch")
    return PileupBatch(b.value)
