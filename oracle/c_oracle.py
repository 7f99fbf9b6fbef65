"""ORACLE — ctypes front end of oracle/spg_oracle.c (test infrastructure only).

Builds ``oracle/_build/libspg_oracle.so`` on demand (``make -C oracle``).  Same
normalised outputs as ``reference_port.OracleCaller`` so the two restatements and
the golden vectors can be compared with one helper (tests/oracle_util.py).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "libspg_oracle.so")
NIBBLE = "=ACMGRSVTWYHKDBN"

VARIANT_DTYPE = np.dtype([("start", "<i8"), ("dp", "<i4"), ("ad", "<i4"), ("pl", "<i4"), ("score", "<i4"),
                          ("ref", "u1"), ("alt", "u1"), ("gl_zero", "u1"), ("pad", "u1", 5),
                          ("gl", "<f8"), ("gl_linear", "<f8"), ("qual", "<f8")])

_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(os.path.join(HERE, "spg_oracle.c")):
            build()
        L = C.CDLL(LIB)
        L.spo_create.restype = C.c_void_p
        L.spo_create.argtypes = [C.c_int64, C.c_char_p, C.c_int, C.c_int, C.c_int, C.c_double, C.c_void_p]
        L.spo_destroy.argtypes = [C.c_void_p]
        L.spo_reset.argtypes = [C.c_void_p]
        L.spo_accumulate.restype = C.c_int
        L.spo_accumulate.argtypes = [C.c_void_p, C.c_int64, C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p]
        L.spo_finalize.restype = C.c_int64
        L.spo_finalize.argtypes = [C.c_void_p]
        L.spo_n_present.restype = C.c_int64
        L.spo_n_present.argtypes = [C.c_void_p]
        L.spo_memory.argtypes = [C.c_void_p] + [C.c_void_p] * 8
        L.spo_variants.argtypes = [C.c_void_p, C.c_void_p]
        L.spo_variant_size.restype = C.c_int
        L.spo_set_threads.argtypes = [C.c_int]
        L.spo_max_threads.restype = C.c_int
        assert L.spo_variant_size() == VARIANT_DTYPE.itemsize
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


class COracle:
    """Bit-exact C restatement of LiveVariantCaller.process_pileup_column + prepare_variants."""

    def __init__(self, reference: str, minBaseQuality=30, minTotalDepth=10, minAlleleDepth=5,
                 minEvidenceRatio=0.10, eps_lut=None):
        from .reference_port import eps_lut as _eps
        L = lib()
        self.reference = reference
        self.n_pos = len(reference)
        lut = np.asarray(eps_lut if eps_lut is not None else _eps(), dtype=np.float64)
        self._h = L.spo_create(self.n_pos, reference.encode("latin-1"), int(minBaseQuality), int(minTotalDepth),
                               int(minAlleleDepth), float(minEvidenceRatio), _p(lut))
        self.n_var = 0
        self.minTotalDepth = int(minTotalDepth)

    def __del__(self):
        if getattr(self, "_h", None):
            lib().spo_destroy(self._h)
            self._h = None

    def reset(self):
        lib().spo_reset(self._h)

    @staticmethod
    def set_threads(n: int):
        """OpenMP threads of accumulate/finalize (1 = sequential; outputs identical for any count)."""
        lib().spo_set_threads(int(n))

    @staticmethod
    def max_threads() -> int:
        return lib().spo_max_threads()

    def accumulate(self, pos_begin, offsets, codes, quals):
        o = np.ascontiguousarray(offsets, dtype=np.uint64)
        c = np.ascontiguousarray(codes, dtype=np.uint8)
        q = np.ascontiguousarray(quals, dtype=np.uint8)
        rc = lib().spo_accumulate(self._h, int(pos_begin), len(o) - 1, _p(o), _p(c), _p(q))
        if rc != 0:
            raise ValueError(f"spo_accumulate failed ({rc})")

    def finalize(self):
        self.n_var = lib().spo_finalize(self._h)
        return self.n_var

    def memory_arrays(self):
        n = lib().spo_n_present(self._h)
        out = dict(pos=np.zeros(n, np.int64), depth=np.zeros(n, np.uint64), n_del=np.zeros(n, np.uint64),
                   n_skip=np.zeros(n, np.uint64), n_all=np.zeros(n, np.uint8), codes=np.zeros((n, 16), np.uint8),
                   counts=np.zeros((n, 16), np.uint32), gl=np.zeros((n, 16), np.float64))
        lib().spo_memory(self._h, *[_p(out[k]) for k in ("pos", "depth", "n_del", "n_skip", "n_all", "codes",
                                                             "counts", "gl")])
        return out

    def variants_array(self):
        v = np.zeros(self.n_var, VARIANT_DTYPE)
        if self.n_var:
            lib().spo_variants(self._h, _p(v))
        return v

    # ---- normalised views (same shape as reference_port / golden) ----
    def memory_summary(self):
        m = self.memory_arrays()
        out = []
        for i in range(len(m["pos"])):
            p = int(m["pos"][i])
            out.append([p, self.reference[p], int(m["depth"][i]),
                        [[NIBBLE[m["codes"][i, k]], int(m["counts"][i, k])] for k in range(m["n_all"][i])]])
        return out

    def gl_table(self):
        m = self.memory_arrays()
        out = {}
        for i in range(len(m["pos"])):
            if int(m["depth"][i]) >= self.minTotalDepth:
                out[int(m["pos"][i])] = {NIBBLE[m["codes"][i, k]]: float(m["gl"][i, k]) for k in range(m["n_all"][i])}
        return out

    def variants(self):
        out = []
        for r in self.variants_array():
            gl = 0 if r["gl_zero"] else float(r["gl"])
            out.append({"start": int(r["start"]), "stop": int(r["start"]) + 1,
                        "alleles": (chr(r["ref"]), chr(r["alt"])), "qual": float(r["qual"]),
                        "info": {"DP": int(r["dp"]), "AD": int(r["ad"]), "GL": gl, "PL": int(r["pl"]),
                                 "SCORE": int(r["score"])}})
        return out
