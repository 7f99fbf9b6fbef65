"""CPU-side checks of the drop-in boundary: the library builds for gfx950, loads, and exports every
symbol include/spings_gpu.h declares, with the struct layouts the ctypes shim assumes.  No compute
calls (no GPU here)."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared(header):
    txt = open(os.path.join(ROOT, "include", header)).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(spg_[a-z_0-9]+)\s*\(", txt) + re.findall(r"\b(spp_[a-z_0-9]+)\s*\(", txt)))


@pytest.fixture(scope="module")
def gpu_lib_path():
    import spings  # noqa: F401
    from covid_spings_variant_caller_amd import build
    return build.build_gpu()


def test_gpu_library_exports_every_declared_symbol(gpu_lib_path):
    lib = ctypes.CDLL(gpu_lib_path)
    names = _declared("spings_gpu.h")
    assert len(names) >= 20
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    out = subprocess.run(["nm", "-D", "--defined-only", gpu_lib_path], capture_output=True, text=True).stdout
    for n in names:
        assert re.search(rf"\bT {n}\b", out), n


def test_struct_layouts_match_shim(gpu_lib_path):
    from covid_spings_variant_caller_amd import _native as N
    L = N.gpu_lib()
    assert L.spg_sizeof_candidate() == N.CANDIDATE_DTYPE.itemsize == 56
    assert L.spg_sizeof_detail() == N.DETAIL_DTYPE.itemsize == 224
    assert L.spg_sizeof_acc() == 160
    assert ctypes.sizeof(N.SpgParams) == 56
    assert L.spg_abi_version() == 1


def test_code_object_targets_gfx950(gpu_lib_path):
    data = open(gpu_lib_path, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data          # embedded offload bundle id


def test_errors_are_reported_without_gpu(gpu_lib_path):
    from covid_spings_variant_caller_amd import _native as N
    L = N.gpu_lib()
    assert L.spg_reset(None) != 0
    assert b"null" in L.spg_last_error()


def test_pileup_library_exports_every_declared_symbol():
    import spings  # noqa: F401
    from covid_spings_variant_caller_amd import build
    from covid_spings_variant_caller_amd import _native as N
    path = build.build_pileup()
    lib = ctypes.CDLL(path)
    names = _declared("spings_pileup.h")
    assert len(names) >= 10
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    assert ctypes.sizeof(N.SppParams) == 40


def test_hot_kernels_do_not_spill_to_scratch():
    """The build records hipcc's kernel-resource-usage remarks (_lib/kernel_resources.json): no kernel
    on a measured path may spill to scratch (a spill there cost 60 % of the deep kernel's speed once),
    and the deep accumulate keeps 4 waves per SIMD (16 per CU, the LDS limit)."""
    import json
    import os
    from covid_spings_variant_caller_amd import build as B
    path = os.path.join(B.LIBDIR, "kernel_resources.json")
    if not os.path.exists(path):
        pytest.skip("library built without the resource record")
    res = json.load(open(path))
    hot = {k: v for k, v in res.items() if any(h in k for h in B.HOT_KERNELS)}
    assert hot, res
    assert all(v.get("scratch", 0) == 0 for v in hot.values()), {k: v for k, v in hot.items() if v.get("scratch")}
    deep = [v for k, v in hot.items() if k.startswith("spg::k_acc_seg<4, true, 4")]
    assert deep and all(v["waves_per_simd"] >= 4 for v in deep), deep


def test_python_modules_import():
    """Every package module imports on a CPU host (no GPU calls at import)."""
    import importlib
    for m in ("engine", "live_variant_caller", "multi", "shard", "pileup", "synth"):
        importlib.import_module(f"covid_spings_variant_caller_amd.{m}")
