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
