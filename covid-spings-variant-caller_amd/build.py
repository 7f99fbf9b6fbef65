"""Build the native libraries in-tree (gfx950).

* ``_lib/libspings_gpu.so``    — HIP kernels + C-ABI (include/spings_gpu.h), hipcc --offload-arch=gfx950
* ``_lib/libspings_pileup.so`` — host C++ BAM/SAM reader + htslib-faithful pileup (include/spings_pileup.h)

The .so files are git-ignored but travel to the GPU box with the gpurun snapshot.
"""
from __future__ import annotations

import json
import os
import re
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIBDIR = os.path.join(PKG, "_lib")
INC = os.path.join(ROOT, "include")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

GPU_SOURCES = ["spg_kernels.hip", "spg_tile.hip", "spg_lite.hip", "spg_fill.hip", "spg_inflate.hip", "spg_ckpt.hip", "spg_bam.hip", "spg_plan.hip", "spg_api.cpp", "spg_multi.cpp"]
GPU_HEADERS = ["spg_device.h", "spg_common.h"]
PILEUP_SOURCES = ["spp_pileup.cpp"]


def _digest(deps, cmd) -> str:
    """Content hash of a build step: its inputs' bytes and its command line."""
    import hashlib
    h = hashlib.sha256(" ".join(cmd).encode())
    for d in deps:
        with open(d, "rb") as f:
            h.update(os.path.basename(d).encode() + b"\0" + f.read())
    return h.hexdigest()


def _stale(out, deps, cmd=()):
    """An output is rebuilt when it is missing or when its recorded input hash (`<out>.sha256`) differs from the
    inputs' and command's now: content, not mtimes (the snapshot that travels to the GPU box keeps mtimes it did
    not produce)."""
    if not os.path.exists(out) or not os.path.exists(out + ".sha256"):
        return True
    with open(out + ".sha256") as f:
        return f.read().strip() != _digest(deps, cmd)


def _stamp(out, deps, cmd=()):
    with open(out + ".sha256", "w") as f:
        f.write(_digest(deps, cmd))


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return r


def build_gpu(force=False, verbose=False) -> str:
    """One object per source, compiled in parallel (each a separate hipcc; the sources share no device code),
    then linked: a kernel edit rebuilds one object."""
    from concurrent.futures import ThreadPoolExecutor
    os.makedirs(LIBDIR, exist_ok=True)
    objdir = os.path.join(LIBDIR, "obj")
    os.makedirs(objdir, exist_ok=True)
    out = os.path.join(LIBDIR, "libspings_gpu.so")
    hdrs = [os.path.join(CSRC, f) for f in GPU_HEADERS] + [os.path.join(INC, "spings_gpu.h")]
    base = [HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", f"-I{INC}"]
    jobs = []
    for f in GPU_SOURCES:
        src, obj = os.path.join(CSRC, f), os.path.join(objdir, f + ".o")
        if force or _stale(obj, [src] + hdrs, base):
            jobs.append(base + ["-c", src, "-o", obj + ".tmp", "-Rpass-analysis=kernel-resource-usage"])
    objs = [os.path.join(objdir, f + ".o") for f in GPU_SOURCES]

    def compile_one(cmd):
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        r = _run(cmd)
        obj = cmd[-2][:-4]
        os.replace(cmd[-2], obj)
        src = cmd[cmd.index("-c") + 1]
        _stamp(obj, [src] + hdrs, base)
        return r.stderr

    res_path = os.path.join(LIBDIR, "kernel_resources.json")
    if jobs:
        with ThreadPoolExecutor(min(len(jobs), max(1, (os.cpu_count() or 2)))) as ex:
            remarks = list(ex.map(compile_one, jobs))
        res = {}
        if os.path.exists(res_path) and len(jobs) < len(GPU_SOURCES):
            with open(res_path) as fh:
                res = json.load(fh)
        new = kernel_resources("\n".join(remarks))
        # (kernels of the recompiled sources replace their old entries)
        rebuilt = {os.path.basename(j[j.index("-c") + 1]) for j in jobs}
        res = {k: v for k, v in res.items() if v.get("src") not in rebuilt}
        for j, rem in zip(jobs, remarks):
            for k, v in kernel_resources(rem).items():
                v["src"] = os.path.basename(j[j.index("-c") + 1])
                res[k] = v
        with open(res_path, "w") as fh:
            json.dump(res, fh, indent=1, sort_keys=True)
        for k, v in new.items():
            if v.get("scratch", 0) and any(h in k for h in HOT_KERNELS):
                print(f"WARNING: hot kernel {k} spills to scratch ({v['scratch']} B/lane)", file=sys.stderr)
    # (-z defs: a kernel launcher the C-ABI declares but no source defines fails the build, not the load)
    cmd = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-Wl,-z,defs", "-o", out + ".tmp"] + objs + ["-lrccl"]
    if force or jobs or _stale(out, objs, cmd):
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        _run(cmd)
        os.replace(out + ".tmp", out)
        _stamp(out, objs, cmd)
    return out


# kernels on the measured paths: a scratch spill there costs occupancy and time (tests/test_cabi.py)
HOT_KERNELS = ("k_acc_seg<4", "k_acc_tile", "k_acc_lite", "k_fold_hist", "k_fill", "k_f2_", "k_finalize", "k_inflate", "k_bam_")


def kernel_resources(remarks: str) -> dict:
    """Per-kernel VGPRs / SGPR spills / scratch / occupancy / LDS from hipcc's kernel-resource-usage
    remarks (demangled names)."""
    out, cur = {}, None
    for line in remarks.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            name = m.group(1)
            try:
                name = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip() or name
            except OSError:
                pass
            cur = out.setdefault(name.split("(")[0].replace("void ", ""), {})
            continue
        if cur is None:
            continue
        for key, pat in (("vgpr", r"VGPRs: (\d+)"), ("sgpr_spill", r"SGPRs Spill: (\d+)"),
                         ("vgpr_spill", r"VGPRs Spill: (\d+)"), ("scratch", r"ScratchSize \[bytes/lane\]: (\d+)"),
                         ("waves_per_simd", r"Occupancy \[waves/SIMD\]: (\d+)"), ("lds", r"LDS Size \[bytes/block\]: (\d+)")):
            m = re.search(pat, line)
            if m:
                cur[key] = int(m.group(1))
    return out


def build_pileup(force=False, verbose=False) -> str:
    os.makedirs(LIBDIR, exist_ok=True)
    out = os.path.join(LIBDIR, "libspings_pileup.so")
    srcs = [os.path.join(CSRC, f) for f in PILEUP_SOURCES]
    if not all(os.path.exists(s) for s in srcs):
        return ""
    deps = srcs + [os.path.join(INC, "spings_pileup.h"), os.path.join(INC, "spings_gpu.h")]
    cxx = shutil.which("g++") or "g++"
    cmd = [cxx, "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", f"-I{INC}", "-o", out + ".tmp"] + srcs + ["-lz", "-ldl", "-pthread"]
    if force or _stale(out, deps, cmd):
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        _run(cmd)
        os.replace(out + ".tmp", out)
        _stamp(out, deps, cmd)
    return out


def build_all(force=False, verbose=False):
    return build_gpu(force, verbose), build_pileup(force, verbose)


if __name__ == "__main__":
    print(build_all(force="--force" in sys.argv or os.environ.get("SPG_FORCE_BUILD") == "1", verbose=True))
