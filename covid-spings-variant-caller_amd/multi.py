"""MultiEngine — the C-ABI's one-process multi-device context (include/spings_gpu.h spg_multi_*): each device
owns a coordinate range, host batches are sliced at the cuts, and the call tables come back with one RCCL
gather.  The torch-free counterpart of shard.ShardedEngine (one process per GPU over torch.distributed)."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _native as N
from .engine import eps_lut


class MultiEngine:
    def __init__(self, devices, n_pos: int, min_base_quality: int = 30, min_total_depth: int = 10,
                 min_allele_depth: int = 5, min_evidence_ratio: float = 0.10, reference: str | None = None,
                 calls_only: bool = True):
        self._L = N.gpu_lib()
        self.devices = [int(d) for d in devices]
        self.n_pos = int(n_pos)
        self.params = N.SpgParams(int(min_base_quality), int(min_total_depth), int(min_allele_depth),
                                  N.SPG_P_CALLS_ONLY if calls_only else 0, float(min_evidence_ratio))
        devs = (C.c_int * len(self.devices))(*self.devices)
        h = C.c_void_p()
        self._check(self._L.spg_multi_create(devs, len(self.devices), self.n_pos, C.byref(self.params), C.byref(h)),
                    "spg_multi_create")
        self._h = h
        self._lut = eps_lut()
        self._check(self._L.spg_multi_set_eps_lut(self._h, N.ptr(self._lut)), "spg_multi_set_eps_lut")
        if reference is not None:
            self.set_reference(reference)

    def _check(self, rc, what):
        if rc != 0:
            raise RuntimeError(f"{what}: {self._L.spg_multi_last_error().decode()}")

    def close(self):
        if getattr(self, "_h", None):
            self._L.spg_multi_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_reference(self, seq: str):
        b = seq.encode("latin-1")
        self._check(self._L.spg_multi_set_reference(self._h, b, len(b)), "spg_multi_set_reference")

    def reset(self):
        self._check(self._L.spg_multi_reset(self._h), "spg_multi_reset")

    def accumulate(self, pos_begin: int, offsets, codes, quals):
        o = np.ascontiguousarray(offsets, dtype=np.uint64)
        c = np.ascontiguousarray(codes, dtype=np.uint8)
        q = np.ascontiguousarray(quals, dtype=np.uint8)
        self._check(self._L.spg_multi_accumulate(self._h, int(pos_begin), len(o) - 1, N.ptr(o), N.ptr(c), N.ptr(q),
                                                 len(c), 0), "spg_multi_accumulate")

    def finalize(self):
        self._check(self._L.spg_multi_finalize(self._h), "spg_multi_finalize")

    def partition(self) -> np.ndarray:
        cuts = np.zeros(len(self.devices) + 1, np.int64)
        self._check(self._L.spg_multi_partition(self._h, cuts.ctypes.data_as(C.POINTER(C.c_int64))), "spg_multi_partition")
        return cuts

    def candidates(self) -> np.ndarray:
        """The merged call table in memory order (first_batch, pos, allele rank)."""
        n = C.c_int64()
        cap = 1024
        while True:
            arr = np.zeros(cap, N.CANDIDATE_DTYPE)
            rc = self._L.spg_multi_get_candidates(self._h, N.ptr(arr), cap, C.byref(n))
            if rc == 0:
                return arr[:n.value]
            if n.value <= cap:
                self._check(rc, "spg_multi_get_candidates")
            cap = int(n.value)
