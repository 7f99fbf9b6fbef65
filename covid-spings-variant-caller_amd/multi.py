"""MultiEngine — the C-ABI's one-process multi-device context (include/spings_gpu.h spg_multi_*): each device
owns a coordinate range (its own context over that range only), host batches and BAM records plans are sliced at
the cuts (the device pileup runs on every device), cuts follow the entries and are re-planned when the load drifts,
and the call tables come back with one RCCL gather.  The torch-free counterpart of shard.ShardedEngine (one
process per GPU over torch.distributed), and the engine behind LiveVariantCaller(..., devices=[...]): it offers
the PileupEngine methods the caller uses (accumulate, accumulate_bam_records, finalize, variants, table, history)
with positions in reference coordinates."""
from __future__ import annotations

import ctypes as C
import threading
from typing import Dict, List

import numpy as np

from . import _native as N
from .engine import PileupEngine, eps_lut


def plan_cuts(weights, bucket: int, n_pos: int, n: int) -> np.ndarray:
    """spg_multi_plan_cuts: equal-entry cuts over a bucket histogram (host only)."""
    w = np.ascontiguousarray(weights, dtype=np.uint64)
    cuts = np.zeros(n + 1, np.int64)
    rc = N.gpu_lib().spg_multi_plan_cuts(N.ptr(w) if len(w) else None, len(w), int(bucket), int(n_pos), int(n),
                                         cuts.ctypes.data_as(C.POINTER(C.c_int64)))
    if rc != 0:
        raise RuntimeError(f"spg_multi_plan_cuts: {N.gpu_lib().spg_multi_last_error().decode()}")
    return cuts


class TableRetry(RuntimeError):
    """spg_multi_wait_candidates returned 1: a device's table did not fit its copy (the copies grow from the tables
    seen) or carried an error word; the sample's table must be taken synchronously before its reset."""


class MultiEngine:
    def __init__(self, devices, n_pos: int, min_base_quality: int = 30, min_total_depth: int = 10,
                 min_allele_depth: int = 5, min_evidence_ratio: float = 0.10, reference: str | None = None,
                 calls_only: bool = True):
        self._L = N.gpu_lib()
        self._lock = threading.RLock()
        self.devices = [int(d) for d in devices]
        self.n_pos = int(n_pos)
        self.calls_only = bool(calls_only)
        self.params = N.SpgParams(int(min_base_quality), int(min_total_depth), int(min_allele_depth),
                                  N.SPG_P_CALLS_ONLY if calls_only else 0, float(min_evidence_ratio))
        devs = (C.c_int * len(self.devices))(*self.devices)
        h = C.c_void_p()
        self._check(self._L.spg_multi_create(devs, len(self.devices), self.n_pos, C.byref(self.params), C.byref(h)),
                    "spg_multi_create")
        self._h = h
        self._lut = eps_lut()
        self._check(self._L.spg_multi_set_eps_lut(self._h, N.ptr(self._lut)), "spg_multi_set_eps_lut")
        self._seq = 0
        self.reference = None
        if reference is not None:
            self.set_reference(reference)

    def _check(self, rc, what):
        if rc != 0:
            raise N.NativeError(f"{what}: {self._L.spg_multi_last_error().decode()}")

    def close(self):
        with self._lock:
            if getattr(self, "_h", None):
                self._L.spg_multi_destroy(self._h)
                self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- lifecycle / input ---------------------------------------------------------------------
    def set_reference(self, seq: str):
        with self._lock:
            b = seq.encode("latin-1") if isinstance(seq, str) else bytes(seq)
            self._check(self._L.spg_multi_set_reference(self._h, b, len(b)), "spg_multi_set_reference")
            self.reference = seq

    def reset(self):
        with self._lock:
            self._check(self._L.spg_multi_reset(self._h), "spg_multi_reset")

    def set_rebalance(self, ratio: float, max_batches: int):
        with self._lock:
            self._check(self._L.spg_multi_set_rebalance(self._h, float(ratio), int(max_batches)), "spg_multi_set_rebalance")

    def replans(self) -> int:
        n = C.c_int64()
        with self._lock:
            self._check(self._L.spg_multi_replans(self._h, C.byref(n)), "spg_multi_replans")
        return n.value

    def accumulate(self, pos_begin: int, offsets, codes, quals, trusted: bool = False, **_):
        with self._lock:
            o = np.ascontiguousarray(offsets, dtype=np.uint64)
            c = np.ascontiguousarray(codes, dtype=np.uint8)
            q = np.ascontiguousarray(quals, dtype=np.uint8)
            self._check(self._L.spg_multi_accumulate(self._h, int(pos_begin), len(o) - 1, N.ptr(o), N.ptr(c), N.ptr(q),
                                                     len(c), N.SPG_IN_TRUSTED if trusted else 0), "spg_multi_accumulate")
            self._seq += 1

    def plan(self, pos_begin: int, offsets) -> np.ndarray:
        """The cuts (n + 1 reference positions) a batch with these host offsets gets (spg_multi_plan): the sample's
        cuts, planned now from this batch when the sample has none yet."""
        o = np.ascontiguousarray(offsets, dtype=np.uint64)
        cuts = np.zeros(len(self.devices) + 1, np.int64)
        with self._lock:
            self._check(self._L.spg_multi_plan(self._h, int(pos_begin), len(o) - 1, N.ptr(o),
                                               cuts.ctypes.data_as(C.POINTER(C.c_int64))), "spg_multi_plan")
        return cuts

    def prepare_slices(self, pos_begin: int, offsets, slices) -> np.ndarray:
        """The spg_batch descriptors accumulate_slices passes for these slices (a caller that accumulates the same
        resident slices again — a benchmark loop — prepares them once)."""
        o = np.ascontiguousarray(offsets, dtype=np.uint64)
        arr = np.zeros(len(self.devices), N.BATCH_DTYPE)
        for d, s in enumerate(slices):
            if s is None:
                continue
            pb, off, codes, quals = s
            arr[d] = (int(pb), int(off.numel()) - 1, int(off.data_ptr()), int(codes.data_ptr()), int(quals.data_ptr()),
                      int(self._slice_entries(d, pb, off, o, pos_begin)))
        return arr

    def accumulate_slices(self, pos_begin: int, offsets, slices, borrow: bool = True):
        """A batch resident in HBM, one slice per device at the plan's cuts (spg_multi_accumulate_slices):
        slices[d] = (pos_begin, offsets, codes, quals) as device tensors on devices[d] (offsets rebased to 0; None
        where the batch misses the device's range), or prepare_slices' array.  ``offsets``: the whole batch's CSR on
        the host."""
        o = np.ascontiguousarray(offsets, dtype=np.uint64)
        arr = slices if isinstance(slices, np.ndarray) else self.prepare_slices(pos_begin, o, slices)
        flags = N.SPG_IN_DEVICE | (N.SPG_IN_BORROW if borrow else 0)
        with self._lock:
            self._check(self._L.spg_multi_accumulate_slices(self._h, int(pos_begin), len(o) - 1, N.ptr(o), N.ptr(arr),
                                                            flags), "spg_multi_accumulate_slices")
            self._seq += 1

    @staticmethod
    def _slice_entries(d, pb, off, o, pos_begin):
        """Entries of the slice starting at reference position pb with off.numel() - 1 columns (from the host CSR)."""
        a = int(pb) - int(pos_begin)
        return int(o[a + int(off.numel()) - 1]) - int(o[a])

    def accumulate_bam_records(self, batch):
        """A records plan (pileup.AlignmentFile.pileup_records) sharded over the devices: each decodes the reads that
        reach its range (spg_multi_accumulate_records).  Keep ``batch`` open until wait_ticket(input_ticket())."""
        r = batch.records()
        with self._lock:
            self._check(self._L.spg_multi_accumulate_records(self._h, C.byref(r), 0), "spg_multi_accumulate_records")
            self._seq += 1

    def input_ticket(self) -> int:
        return self._seq

    def wait_ticket(self, ticket: int):
        """Every input copy enqueued so far has landed (a ticket waits for all of them: coarser than PileupEngine's)."""
        if ticket:
            self.wait_input()

    def wait_input(self):
        with self._lock:
            self._check(self._L.spg_multi_wait_input(self._h), "spg_multi_wait_input")

    def finalize(self):
        with self._lock:
            self._check(self._L.spg_multi_finalize(self._h), "spg_multi_finalize")

    def sync(self):
        with self._lock:
            for ctx in self._contexts():
                N.check(self._L.spg_sync(ctx), "spg_sync")

    def set_timing(self, level: int):
        with self._lock:
            for ctx in self._contexts():
                N.check(self._L.spg_set_timing(ctx, int(level)), "spg_set_timing")

    def kernel_times(self, cap: int = 4096):
        """Per device: (accumulate ms, finalize ms) of every finalize step since the last call (spg_kernel_times)."""
        out = []
        with self._lock:
            for ctx in self._contexts():
                a, f = np.zeros(cap, np.float32), np.zeros(cap, np.float32)
                n = C.c_int64()
                N.check(self._L.spg_kernel_times(ctx, N.ptr(a), N.ptr(f), cap, C.byref(n)), "spg_kernel_times")
                out.append((a[:n.value].copy(), f[:n.value].copy()))
        return out

    # -- results ---------------------------------------------------------------------------------
    def partition(self) -> np.ndarray:
        cuts = np.zeros(len(self.devices) + 1, np.int64)
        with self._lock:
            self._check(self._L.spg_multi_partition(self._h, cuts.ctypes.data_as(C.POINTER(C.c_int64))),
                        "spg_multi_partition")
        return cuts

    def candidates(self) -> np.ndarray:
        """The merged call table in memory order (first_batch, pos, allele rank), reference positions."""
        n = C.c_int64()
        cap = 1024
        with self._lock:
            while True:
                arr = np.zeros(cap, N.CANDIDATE_DTYPE)
                rc = self._L.spg_multi_get_candidates(self._h, N.ptr(arr), cap, C.byref(n))
                if rc == 0:
                    return arr[:n.value]
                if n.value <= cap:
                    self._check(rc, "spg_multi_get_candidates")
                cap = int(n.value)

    def candidates_async(self) -> int:
        """Enqueue the merged call table without waiting (spg_multi_get_candidates_async): the ticket for
        wait_candidates.  The next sample's reset / accumulate / finalize may go out before that wait."""
        t = C.c_uint64()
        with self._lock:
            self._check(self._L.spg_multi_get_candidates_async(self._h, C.byref(t)), "spg_multi_get_candidates_async")
        return t.value

    def wait_candidates(self, ticket: int) -> np.ndarray:
        """The table a ticket names (spg_multi_wait_candidates), merged in memory order.  Raises TableRetry when a
        device's table outgrew its copy (take that sample's table with candidates() before its reset)."""
        n = C.c_int64()
        with self._lock:
            while True:
                buf = getattr(self, "_wait_buf", None)         # (reused: one host buffer per engine)
                if buf is None:
                    buf = self._wait_buf = np.empty(1024, N.CANDIDATE_DTYPE)
                rc = self._L.spg_multi_wait_candidates(self._h, int(ticket), N.ptr(buf), len(buf), C.byref(n))
                if rc == 0:
                    return buf[:n.value].copy()
                if rc == 1:
                    raise TableRetry(self._L.spg_multi_last_error().decode())
                if n.value <= len(buf):
                    self._check(rc, "spg_multi_wait_candidates")
                self._wait_buf = np.empty(int(n.value), N.CANDIDATE_DTYPE)

    def variants(self) -> List[dict]:
        """The list prepare_variants() returns (live_variant_caller.py:170-185)."""
        return PileupEngine._variants_of(self.candidates())

    def _contexts(self):
        out = []
        for i in range(len(self.devices)):
            h = C.c_void_p()
            if self._L.spg_multi_context(self._h, i, C.byref(h)) != 0:
                return []
            out.append(h)
        return out

    def _cuts_of_contexts(self):
        """The ranges the device contexts cover (the last planned sample's cuts)."""
        try:
            return self.partition()
        except N.NativeError:
            return None

    def table(self) -> Dict[str, np.ndarray]:
        """Every device's per-position table, concatenated in reference coordinates (spg_get_table per device)."""
        n = self.n_pos
        out = dict(depth=np.zeros(n, np.uint32), counts=np.zeros((n, N.SPG_NCOUNT), np.uint32),
                   gl=np.zeros((n, N.SPG_NSLOT), np.float64), flags=np.zeros(n, np.uint8),
                   order=np.zeros(n, np.uint32), first_batch=np.zeros(n, np.uint32))
        with self._lock:
            ctxs, cuts = self._contexts(), self._cuts_of_contexts()
            if not ctxs or cuts is None:
                return out
            for d, ctx in enumerate(ctxs):
                lo, hi = int(cuts[d]), int(cuts[d + 1])
                N.check(self._L.spg_get_table(ctx, 0, hi - lo, *[N.ptr(out[k][lo:hi]) for k in
                                                                  ("depth", "counts", "gl", "flags", "order",
                                                                   "first_batch")]), "spg_get_table")
        return out

    def position_entries(self, pos: int, upto=None):
        """(codes, quals) of every entry at reference position ``pos`` (over the first ``upto`` batches), from the device
        whose range holds it."""
        with self._lock:
            ctxs, cuts = self._contexts(), self._cuts_of_contexts()
            if not ctxs or cuts is None:
                return np.zeros(0, np.uint8), np.zeros(0, np.uint8)
            d = int(np.searchsorted(cuts[1:-1], pos, side="right"))
            local = int(pos) - int(cuts[d])
            n = C.c_int64()
            ub = (1 << 62) if upto is None else int(upto)
            N.check(self._L.spg_position_entries_upto(ctxs[d], local, ub, None, None, 0, C.byref(n)),
                    "spg_position_entries")
            codes, quals = np.zeros(n.value, np.uint8), np.zeros(n.value, np.uint8)
            if n.value:
                N.check(self._L.spg_position_entries_upto(ctxs[d], local, ub, N.ptr(codes), N.ptr(quals), n.value,
                                                          C.byref(n)), "spg_position_entries")
        return codes, quals

    def history_count(self) -> int:
        with self._lock:
            ctxs = self._contexts()
            if not ctxs:
                return 0
            n = C.c_int64()
            N.check(self._L.spg_history_count(ctxs[0], C.byref(n)), "spg_history_count")
            return n.value

    def history(self, start: int = 0, min_bq=None):
        """The accumulated batches, reassembled from the devices' slices in reference coordinates:
        [(pos_begin, offsets, codes, quals)] (a batch's extent spans the slices that hold entries)."""
        return list(self.iter_history(start, min_bq))

    def iter_history(self, start: int = 0, min_bq=None):
        """history() one batch at a time; min_bq: each device compacts its slice as the checkpoint keeps it
        (spg_history_copy_compact) before the slices are reassembled."""
        with self._lock:
            ctxs, cuts = self._contexts(), self._cuts_of_contexts()
            n_hist = self.history_count() if ctxs and cuts is not None else 0
        for i in range(max(0, int(start)), n_hist):
            parts = []
            with self._lock:
                for d, ctx in enumerate(ctxs):
                    pb, nc, ne = C.c_int64(), C.c_int64(), C.c_uint64()
                    N.check(self._L.spg_history_info(ctx, i, C.byref(pb), C.byref(nc), C.byref(ne)), "spg_history_info")
                    if ne.value == 0:
                        continue
                    off = np.zeros(nc.value + 1, np.uint64)
                    codes = np.empty(ne.value, np.uint8)
                    quals = np.empty(ne.value, np.uint8)
                    if min_bq is None:
                        N.check(self._L.spg_history_copy(ctx, i, N.ptr(off), N.ptr(codes), N.ptr(quals)),
                                "spg_history_copy")
                    else:
                        k = C.c_uint64()
                        N.check(self._L.spg_history_copy_compact(ctx, i, int(min_bq), N.ptr(off), N.ptr(codes),
                                                                 N.ptr(quals), C.byref(k)), "spg_history_copy_compact")
                        codes, quals = codes[:k.value], quals[:k.value]
                    parts.append((int(cuts[d]) + pb.value, off, codes, quals))
            if not parts:
                yield (0, np.zeros(1, np.uint64), np.zeros(0, np.uint8), np.zeros(0, np.uint8))
                continue
            p0 = parts[0][0]
            p1 = parts[-1][0] + len(parts[-1][1]) - 1
            lens = np.zeros(p1 - p0, np.int64)
            for pb, off, _, _ in parts:
                lens[pb - p0:pb - p0 + len(off) - 1] = np.diff(off.astype(np.int64))
            offs = np.zeros(p1 - p0 + 1, np.uint64)
            np.cumsum(lens, out=offs[1:])
            yield (p0, offs, np.concatenate([p[2] for p in parts]), np.concatenate([p[3] for p in parts]))
