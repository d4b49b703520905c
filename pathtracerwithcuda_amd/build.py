"""Build recipe for libpt_hip.so (HIP kernels for gfx950 + host C++), in-tree.

Every float expression of the hot path must round exactly as the C oracle's does, so both the
device and host halves are compiled with -ffp-contract=off and without fast-math (DESIGN.md
§Numerics). Run `python -m pathtracerwithcuda_amd.build` or call build().
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
# PT_CSRC / PT_LIBDIR / PT_EXTRA_FLAGS: an alternative build (a patched source copy, compiler-flag A/B runs,
# tools/build_dup.sh); the product is csrc/ built into lib/
CSRC = os.environ.get("PT_CSRC") or os.path.join(HERE, "csrc")
LIBDIR = os.environ.get("PT_LIBDIR") or os.path.join(HERE, "lib")
INCLUDE = os.path.join(os.path.dirname(HERE), "include")
LIB = os.path.join(LIBDIR, "libpt_hip.so")
CLI = os.path.join(LIBDIR, "pt_render")  # headless host program (csrc/pt_cli.cpp) linked against LIB

ARCH = os.environ.get("PT_OFFLOAD_ARCH", "gfx950")
COMMON = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math", "-Wall", "-Wno-unused-function",
          f"-I{INCLUDE}", f"-I{CSRC}"]
# -fno-slp-vectorize: the SLP pass packs independent fp32 lanes into v_pk_* ops that need extra
# v_mov shuffles and 3 more VGPRs; without it pass_kernel_u is 3.6% faster (profiles/r01/ab_slp.txt).
# It does not change a single rounding (no contraction, no reassociation): parity stays bit-exact.
HIP_FLAGS = ["-fno-slp-vectorize"] + os.environ.get("PT_EXTRA_FLAGS", "").split()

HIP_SOURCES = ["pt_kernels.hip", "pt_wavefront.hip", "pt_bvh.hip", "pt_bvh_sah.hip", "pt_runtime.cpp"]
CXX_SOURCES = ["pt_host.cpp", "pt_loader.cpp", "pt_image.cpp", "pt_jpeg.cpp"]
LINK_LIBS = ["-lz"]  # zlib: PNG inflate/deflate (pt_image.cpp)


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the HIP library cannot be built")


def _sources_newer(target: str, sources: list[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(s) > t for s in sources)


def _run(cmd: list[str]) -> None:
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"build failed: {' '.join(cmd)}\n{res.stdout}\n{res.stderr}")


def build(force: bool = False, verbose: bool = False) -> str:
    os.makedirs(LIBDIR, exist_ok=True)
    objdir = os.path.join(LIBDIR, "obj")
    os.makedirs(objdir, exist_ok=True)
    deps = [os.path.join(CSRC, f) for f in os.listdir(CSRC)] + [os.path.join(INCLUDE, f) for f in os.listdir(INCLUDE)]
    if not force and not _sources_newer(LIB, deps) and not _sources_newer(CLI, deps):
        return LIB
    hipcc = _hipcc()
    jobs = []
    objs = []
    for src in HIP_SOURCES:
        obj = os.path.join(objdir, src + ".o")
        objs.append(obj)
        jobs.append([hipcc, "-x", "hip", f"--offload-arch={ARCH}", *COMMON, *HIP_FLAGS, "-c", os.path.join(CSRC, src), "-o", obj])
    for src in CXX_SOURCES:
        obj = os.path.join(objdir, src + ".o")
        objs.append(obj)
        jobs.append(["g++", *COMMON, "-c", os.path.join(CSRC, src), "-o", obj])
    with ThreadPoolExecutor(max_workers=min(len(jobs), 4)) as ex:
        for cmd, _ in zip(jobs, ex.map(_run, jobs)):
            if verbose:
                print(" ".join(cmd), file=sys.stderr)
    tmp = LIB + ".tmp"
    _run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, *LINK_LIBS, "-o", tmp])
    os.replace(tmp, LIB)
    _run(["g++", *COMMON, os.path.join(CSRC, "pt_cli.cpp"), "-o", CLI + ".tmp", f"-L{LIBDIR}", "-lpt_hip",
          "-Wl,-rpath,$ORIGIN"])
    os.replace(CLI + ".tmp", CLI)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
