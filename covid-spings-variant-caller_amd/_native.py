"""ctypes bindings of the two native libraries (include/spings_gpu.h, include/spings_pileup.h).

The GPU library is the only compute path of the engine: if ``_lib/libspings_gpu.so`` is missing
the import of the engine fails loudly (no CPU fallback exists)."""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

PKG = os.path.dirname(os.path.abspath(__file__))
LIBDIR = os.path.join(PKG, "_lib")
GPU_LIB = os.path.join(LIBDIR, "libspings_gpu.so")
PILEUP_LIB = os.path.join(LIBDIR, "libspings_pileup.so")

SPG_NSLOT = 5
SPG_NCOUNT = 8
SPG_CODE_DEL = 16
SPG_CODE_SKIP = 17
SPG_F_PRESENT, SPG_F_EVALUATED, SPG_F_REPLAYED, SPG_F_EXOTIC, SPG_F_CANDIDATE, SPG_F_PARTIAL = 1, 2, 4, 8, 16, 32
SPG_P_CALLS_ONLY = 1
SPG_IN_DEVICE, SPG_IN_BORROW, SPG_IN_TRUSTED = 1, 2, 4
NIBBLE = "=ACMGRSVTWYHKDBN"
SLOT_CHARS = "ACGTN"
SLOT_CODES = (1, 2, 4, 8, 15)


class SpgParams(C.Structure):
    _fields_ = [("min_base_quality", C.c_int32), ("min_total_depth", C.c_int32),
                ("min_allele_depth", C.c_int32), ("flags", C.c_int32),
                ("min_evidence_ratio", C.c_double), ("reserved1", C.c_int64 * 4)]


CANDIDATE_DTYPE = np.dtype([("pos", "<i8"), ("dp", "<i4"), ("ad", "<i4"), ("pl", "<i4"), ("score", "<i4"),
                            ("ref", "u1"), ("alt", "u1"), ("gl_zero", "u1"), ("rank", "u1"),
                            ("first_batch", "<u4"), ("gl", "<f8"), ("gl_linear", "<f8"), ("qual", "<f8")])
# spg_batch (include/spings_gpu.h): one CSR batch of spg_accumulate_batches
BATCH_DTYPE = np.dtype([("pos_begin", "<i8"), ("n_cols", "<i8"), ("offsets", "<u8"), ("base_code", "<u8"),
                        ("qual", "<u8"), ("n_entries", "<u8")])


class SpgRecords(C.Structure):
    """spg_records (include/spings_gpu.h): a records plan's raw BAM bytes + per-read index."""
    _fields_ = [("pos_begin", C.c_int64), ("n_cols", C.c_int64), ("n_entries", C.c_uint64),
                ("offsets", C.c_void_p), ("data", C.c_void_p), ("data_bytes", C.c_uint64), ("n_reads", C.c_int64),
                ("rec", C.c_void_p), ("rpos", C.c_void_p), ("rend", C.c_void_p), ("tweak", C.c_void_p),
                ("n_tweaks", C.c_int64), ("tweak_col", C.c_void_p), ("tweak_qual", C.c_void_p),
                ("orig_qual", C.c_void_p), ("orig_bytes", C.c_uint64), ("max_span", C.c_int64),
                ("pos_origin", C.c_int64), ("reserved", C.c_int64 * 3)]


class SpgBamFilter(C.Structure):
    _fields_ = [("stepper", C.c_int32), ("flag_filter", C.c_uint32), ("min_mapping_quality", C.c_int32),
                ("reserved", C.c_int32)]


class SpgBamReads(C.Structure):
    """spg_bam_reads / spp_read_fields arrays (host), n_reads each."""
    _fields_ = [("pos", C.c_void_p), ("end", C.c_void_p), ("mtid", C.c_void_p), ("mpos", C.c_void_p),
                ("isize", C.c_void_p), ("flag", C.c_void_p), ("l_seq", C.c_void_p), ("name_hash", C.c_void_p)]


class SppReadFields(C.Structure):
    _fields_ = [("n", C.c_int64), ("pos", C.c_void_p), ("end", C.c_void_p), ("mtid", C.c_void_p), ("mpos", C.c_void_p),
                ("isize", C.c_void_p), ("flag", C.c_void_p), ("l_seq", C.c_void_p), ("name_hash", C.c_void_p)]


class SpgBamPlan(C.Structure):
    _fields_ = [("pos_begin", C.c_int64), ("n_cols", C.c_int64), ("n_entries", C.c_uint64), ("offsets", C.c_void_p),
                ("n_kept", C.c_int64), ("kept", C.c_void_p), ("n_pairs", C.c_int64), ("pair_a", C.c_void_p),
                ("pair_b", C.c_void_p), ("pair_col", C.c_void_p), ("pair_orig", C.c_void_p), ("orig_bytes", C.c_uint64),
                ("max_span", C.c_int64), ("reserved", C.c_int64 * 4)]


class SppBamMapInfo(C.Structure):
    _fields_ = [("comp", C.c_void_p), ("comp_bytes", C.c_uint64), ("members", C.c_void_p), ("n_members", C.c_int64),
                ("inflated_bytes", C.c_uint64), ("body", C.c_uint64), ("n_ref", C.c_int32), ("reserved", C.c_int32)]


# the fields spg_bam_reads_copy returns (name, dtype)
BAM_READ_FIELDS = (("pos", np.int32), ("end", np.int32), ("mtid", np.int32), ("mpos", np.int32), ("isize", np.int32),
                   ("flag", np.uint16), ("l_seq", np.uint32), ("name_hash", np.uint64))


DETAIL_DTYPE = np.dtype([("pos", "<i8"), ("depth", "<u4"), ("n_alleles", "u1"), ("pad", "u1", 3),
                         ("code", "u1", 16), ("count", "<u4", 16), ("gl", "<f8", 16)])

_gpu = None
_pileup = None


class NativeError(RuntimeError):
    pass


def _sig(f, res, *args):
    f.restype = res
    f.argtypes = list(args)


def gpu_lib():
    """Load libspings_gpu.so (raises if it has not been built: there is no fallback)."""
    global _gpu
    if _gpu is not None:
        return _gpu
    # One HIP runtime per process: torch ships its own libamdhip64 (same SONAME).  Loading torch
    # first makes our library bind to that already-loaded runtime instead of /opt/rocm's copy
    # (two runtimes in one process leave the second without GPUs).
    try:
        import torch  # noqa: F401
    except Exception:
        pass
    if not os.path.exists(GPU_LIB):
        raise NativeError(f"{GPU_LIB} not found: build it with __graft_entry__.build() "
                          "(python covid-spings-variant-caller_amd/build.py); the engine has no CPU path")
    L = C.CDLL(GPU_LIB)
    vp, i64, u64, i32 = C.c_void_p, C.c_int64, C.c_uint64, C.c_int
    _sig(L.spg_last_error, C.c_char_p)
    _sig(L.spg_abi_version, i32)
    _sig(L.spg_create, i32, i32, i64, C.POINTER(SpgParams), C.POINTER(vp))
    _sig(L.spg_destroy, i32, vp)
    _sig(L.spg_reset, i32, vp)
    _sig(L.spg_set_eps_lut, i32, vp, vp)
    _sig(L.spg_set_reference, i32, vp, C.c_char_p, i64)
    _sig(L.spg_accumulate, i32, vp, i64, i64, vp, vp, vp, u64)
    _sig(L.spg_accumulate_ex, i32, vp, i64, i64, vp, vp, vp, u64, C.c_uint32)
    _sig(L.spg_accumulate_batches, i32, vp, vp, i64, C.c_uint32)
    _sig(L.spg_accumulate_samples, i32, vp, i64, i64, i64, vp, vp, vp, vp, u64, C.c_uint32)
    _sig(L.spg_history_samples, i32, vp, i64, C.POINTER(i64), vp)
    _sig(L.spg_accumulate_records, i32, vp, C.POINTER(SpgRecords), C.c_uint32)
    _sig(L.spg_host_alloc, i32, C.c_size_t, C.POINTER(vp))
    _sig(L.spg_host_free, i32, vp)
    _sig(L.spg_wait_input, i32, vp)
    _sig(L.spg_multi_create, i32, C.POINTER(C.c_int), i32, i64, C.POINTER(SpgParams), C.POINTER(vp))
    _sig(L.spg_multi_destroy, i32, vp)
    _sig(L.spg_multi_last_error, C.c_char_p)
    _sig(L.spg_multi_set_eps_lut, i32, vp, vp)
    _sig(L.spg_multi_set_reference, i32, vp, C.c_char_p, i64)
    _sig(L.spg_multi_reset, i32, vp)
    _sig(L.spg_multi_accumulate, i32, vp, i64, i64, vp, vp, vp, u64, C.c_uint32)
    _sig(L.spg_multi_finalize, i32, vp)
    _sig(L.spg_multi_get_candidates, i32, vp, vp, i64, C.POINTER(i64))
    _sig(L.spg_multi_get_candidates_async, i32, vp, C.POINTER(u64))
    _sig(L.spg_multi_wait_candidates, i32, vp, u64, vp, i64, C.POINTER(i64))
    _sig(L.spg_multi_partition, i32, vp, C.POINTER(i64))
    _sig(L.spg_multi_context, i32, vp, i32, C.POINTER(vp))
    _sig(L.spg_multi_accumulate_records, i32, vp, C.POINTER(SpgRecords), C.c_uint32)
    _sig(L.spg_multi_plan, i32, vp, i64, i64, vp, C.POINTER(i64))
    _sig(L.spg_multi_accumulate_slices, i32, vp, i64, i64, vp, vp, C.c_uint32)
    _sig(L.spg_multi_wait_input, i32, vp)
    _sig(L.spg_multi_set_rebalance, i32, vp, C.c_double, i64)
    _sig(L.spg_multi_replans, i32, vp, C.POINTER(i64))
    _sig(L.spg_multi_plan_cuts, i32, vp, i64, i64, i64, i32, C.POINTER(i64))
    _sig(L.spg_set_history_cap, i32, vp, i64)
    _sig(L.spg_history_resident, i32, vp, C.POINTER(i64), C.POINTER(i64), C.POINTER(i64))
    _sig(L.spg_path_counters, i32, vp, C.POINTER(i64), i64)
    _sig(L.spg_bgzf_inflate, i32, i32, vp, C.c_size_t, vp, i64, vp, C.c_size_t, vp, C.POINTER(C.c_float))
    _sig(L.spg_bgzf_last_error, C.c_char_p)
    _sig(L.spg_bgzf_inflate_check, i32, vp, C.c_size_t, vp, i64, vp, C.c_size_t, vp)
    _sig(L.spg_bgzf_release, i32, i32)
    _sig(L.spg_bgzf_inflate_par_check, i32, vp, C.c_size_t, vp, i64, vp, C.c_size_t, vp, vp)
    _sig(L.spg_bgzf_fallbacks, i32, i32, C.POINTER(i64))
    _sig(L.spg_bam_open, i32, vp, vp, u64, vp, i64, u64, i32, i32, C.POINTER(SpgBamFilter), C.POINTER(i64))
    _sig(L.spg_bam_reads_copy, i32, vp, C.POINTER(SpgBamReads))
    _sig(L.spg_bam_accumulate, i32, vp, C.POINTER(SpgBamPlan), C.c_uint32)
    _sig(L.spg_bam_plan_build, i32, vp, i64, i32, C.POINTER(SpgBamPlan))
    _sig(L.spg_bam_plan_download, i32, vp, C.POINTER(SpgBamPlan), vp, vp, vp, vp, vp, vp)
    _sig(L.spg_bam_inflate_ms, i32, vp, C.POINTER(C.c_float))
    _sig(L.spg_bam_inflate_fallbacks, i32, vp, C.POINTER(i64))
    _sig(L.spg_bam_slot, i32, vp, i32)
    _sig(L.spg_bam_upload, i32, vp, i32, vp, u64, vp, i64)
    _sig(L.spg_bam_release, i32, vp)
    _sig(L.spg_position_entries, i32, vp, i64, vp, vp, i64, C.POINTER(i64))
    _sig(L.spg_position_entries_upto, i32, vp, i64, i64, vp, vp, i64, C.POINTER(i64))
    _sig(L.spg_input_ticket, i32, vp, C.POINTER(u64))
    _sig(L.spg_wait_ticket, i32, vp, u64)
    _sig(L.spg_finalize, i32, vp)
    _sig(L.spg_sync, i32, vp)
    _sig(L.spg_stream, i32, vp, C.POINTER(vp))
    _sig(L.spg_get_table, i32, vp, i64, i64, vp, vp, vp, vp, vp, vp)
    _sig(L.spg_count, i32, vp, C.POINTER(i64), C.POINTER(i64))
    _sig(L.spg_get_candidates, i32, vp, vp, i64, C.POINTER(i64))
    _sig(L.spg_get_details, i32, vp, vp, i64, C.POINTER(i64))
    _sig(L.spg_device_results, i32, vp, C.POINTER(vp), C.POINTER(vp))
    _sig(L.spg_copy_candidates_device, i32, vp, vp, i64)
    _sig(L.spg_copy_table_device, i32, vp, vp, i64, C.POINTER(i64))
    _sig(L.spg_last_kernel_ms, i32, vp, C.POINTER(C.c_float), C.POINTER(C.c_float))
    _sig(L.spg_kernel_times, i32, vp, vp, vp, i64, C.POINTER(i64))
    _sig(L.spg_set_timing, i32, vp, i32)
    _sig(L.spg_history_count, i32, vp, C.POINTER(i64))
    _sig(L.spg_history_info, i32, vp, i64, C.POINTER(i64), C.POINTER(i64), C.POINTER(u64))
    _sig(L.spg_history_copy, i32, vp, i64, vp, vp, vp)
    _sig(L.spg_history_copy_compact, i32, vp, i64, i32, vp, vp, vp, C.POINTER(u64))
    _sig(L.spg_history_copy_packed, i32, vp, i64, i32, vp, vp, C.POINTER(C.c_uint64), vp, vp, vp, i64, C.POINTER(i64))
    _sig(L.spg_device_count, i32, C.POINTER(i32))
    _sig(L.spg_sizeof_candidate, C.c_size_t)
    _sig(L.spg_sizeof_detail, C.c_size_t)
    _sig(L.spg_sizeof_acc, C.c_size_t)
    if L.spg_abi_version() != 1:
        raise NativeError("libspings_gpu.so ABI mismatch")
    if L.spg_sizeof_candidate() != CANDIDATE_DTYPE.itemsize or L.spg_sizeof_detail() != DETAIL_DTYPE.itemsize:
        raise NativeError("libspings_gpu.so struct layout mismatch")
    _gpu = L
    return L


def check(rc: int, what: str = ""):
    if rc != 0:
        msg = gpu_lib().spg_last_error().decode(errors="replace")
        raise NativeError(f"{what}: {msg}" if what else msg)


def ptr(a) -> C.c_void_p:
    """Host numpy array or device torch tensor -> void*."""
    if isinstance(a, np.ndarray):
        return a.ctypes.data_as(C.c_void_p)
    return C.c_void_p(int(a.data_ptr()))


# ------------------------------------------------------------------------------------------------
# libspings_pileup.so (include/spings_pileup.h): host BAM/SAM reader + pileup emulator
# ------------------------------------------------------------------------------------------------
SPP_STEPPER = {"all": 0, "nofilter": 1, "samtools": 2}


class SppParams(C.Structure):
    _fields_ = [("stepper", C.c_int32), ("min_mapping_quality", C.c_int32), ("max_depth", C.c_int32),
                ("ignore_overlaps", C.c_int32), ("flag_filter", C.c_uint32), ("n_threads", C.c_int32),
                ("inflate_device", C.c_int32), ("inflate_min_members", C.c_int32), ("reserved", C.c_int64 * 1)]


class SimParams(C.Structure):
    _fields_ = [("depth", C.c_double), ("read_len", C.c_int32), ("snv_every", C.c_int32), ("q_mean", C.c_double),
                ("q_sd", C.c_double), ("q_min", C.c_int32), ("q_max", C.c_int32), ("del_frac", C.c_double),
                ("ins_frac", C.c_double), ("n_rate", C.c_double), ("seed", C.c_uint64), ("n_threads", C.c_int32),
                ("level", C.c_int32), ("reserved", C.c_int64 * 2)]


def pileup_lib():
    """Load libspings_pileup.so (host-only; raises if it has not been built)."""
    global _pileup
    if _pileup is not None:
        return _pileup
    if not os.path.exists(PILEUP_LIB):
        raise NativeError(f"{PILEUP_LIB} not found: build it with __graft_entry__.build()")
    L = C.CDLL(PILEUP_LIB)
    vp, i64, i32 = C.c_void_p, C.c_int64, C.c_int32
    _sig(L.spp_last_error, C.c_char_p)
    _sig(L.spp_host_inflater, C.c_char_p)
    _sig(L.spp_default_params, None, C.POINTER(SppParams))
    _sig(L.spp_open, C.c_int, C.c_char_p, C.POINTER(vp))
    _sig(L.spp_close, C.c_int, vp)
    _sig(L.spp_n_targets, C.c_int, vp, C.POINTER(i32))
    _sig(L.spp_target, C.c_int, vp, i32, C.POINTER(C.c_char_p), C.POINTER(i64))
    _sig(L.spp_target_id, C.c_int, vp, C.c_char_p, C.POINTER(i32))
    _sig(L.spp_pileup, C.c_int, vp, i32, C.POINTER(SppParams), C.POINTER(vp))
    _sig(L.spp_pileup_region, C.c_int, vp, i32, i64, i64, C.POINTER(SppParams), C.POINTER(vp))
    _sig(L.spp_batch_info, C.c_int, vp, C.POINTER(i64), C.POINTER(i64), C.POINTER(C.c_uint64),
         C.POINTER(i64), C.POINTER(i64))
    _sig(L.spp_batch_arrays, C.c_int, vp, C.POINTER(vp), C.POINTER(vp), C.POINTER(vp))
    _sig(L.spp_batch_free, C.c_int, vp)
    _sig(L.spp_pileup_plan, C.c_int, vp, i32, i64, i64, C.POINTER(SppParams), C.POINTER(vp))
    _sig(L.spp_batch_fill, C.c_int, vp, vp, vp)
    _sig(L.spp_pileup_plan_records, C.c_int, vp, i32, i64, i64, C.POINTER(SppParams), C.POINTER(vp))
    _sig(L.spp_batch_records, C.c_int, vp, C.POINTER(SpgRecords))
    _sig(L.spp_set_host_allocator, C.c_int, vp, vp)
    _sig(L.spp_set_inflater, C.c_int, vp, C.c_int)
    _sig(L.spp_bam_map_open, C.c_int, vp, C.c_int, C.POINTER(vp), C.POINTER(SppBamMapInfo))
    _sig(L.spp_bam_map_close, C.c_int, vp)
    _sig(L.spp_pileup_plan_fields, C.c_int, vp, i32, C.POINTER(SppReadFields), C.POINTER(SppParams), C.POINTER(vp))
    _sig(L.spp_batch_device_plan, C.c_int, vp, C.POINTER(SpgBamPlan))
    _sig(L.spp_default_sim_params, None, C.POINTER(SimParams))
    _sig(L.spp_simulate_bam, C.c_int, C.c_char_p, C.c_char_p, C.c_char_p, i64, C.POINTER(SimParams),
         C.POINTER(i64))
    _sig(L.spp_synth_batch, C.c_int, C.c_char_p, i64, i64, i64, C.POINTER(SimParams), i64, C.POINTER(vp))
    _pileup = L
    return L


_pinned_records = False


def use_pinned_records():
    """Route the records plans' host buffers through spg_host_alloc / spg_host_free (pinned: the copy of the
    inflated BAM to HBM is then a DMA without a staging copy).  Idempotent."""
    global _pinned_records
    if _pinned_records:
        return
    G, P = gpu_lib(), pileup_lib()
    pcheck(P.spp_set_host_allocator(C.cast(G.spg_host_alloc, C.c_void_p), C.cast(G.spg_host_free, C.c_void_p)),
           "spp_set_host_allocator")
    _pinned_records = True


_inflater_set = False


def register_gpu_inflater():
    """Register spg_bgzf_inflate as the records plans' BGZF inflater (spp_set_inflater).  Registering does not turn it
    on: each plan selects it through its own parameters (PileupParams.inflate_device), so callers with different
    choices do not override one another.  Idempotent."""
    global _inflater_set
    if _inflater_set:
        return
    G, P = gpu_lib(), pileup_lib()
    pcheck(P.spp_set_inflater(C.cast(G.spg_bgzf_inflate, C.c_void_p), 0), "spp_set_inflater")
    _inflater_set = True


def pcheck(rc: int, what: str = ""):
    if rc != 0:
        msg = pileup_lib().spp_last_error().decode(errors="replace")
        raise NativeError(f"{what}: {msg}" if what else msg)
