#!/usr/bin/env python3
"""Build the framework's native extension `_C.so` in-tree (no hipify, no JIT cache).

Every `csrc/kernels/*.hip` file is compiled by `hipcc --offload-arch=gfx950` straight from
CDNA4 source; `csrc/cpu/*.cpp` (the offload AdamW, packing helpers) and `csrc/comm/*.hip`
are compiled alongside, and everything is linked against libtorch into
`lambda-labs_distributed-training-guide_amd/_C.so`, which `dtg.ops` loads with
`torch.ops.load_library`.  Operator schemas are declared in Python (`dtg/ops/_schema.py`);
the objects here only register implementations (`TORCH_LIBRARY_IMPL(dtg, CUDA|CPU, ...)`).

Incremental: an object is rebuilt when its source or any header under csrc/ is newer.
Usage: python csrc/build.py [-j N] [--force] [--verbose]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
PKG = os.path.join(ROOT, "lambda-labs_distributed-training-guide_amd")
OUT = os.path.join(PKG, "_C.so")
BUILD = os.path.join(ROOT, "build", "obj")
ARCH = os.environ.get("DTG_OFFLOAD_ARCH", "gfx950")


def _torch_paths():
    import torch

    tdir = os.path.dirname(torch.__file__)
    inc = [os.path.join(tdir, "include"), os.path.join(tdir, "include", "torch", "csrc", "api", "include")]
    return tdir, inc, int(torch._C._GLIBCXX_USE_CXX11_ABI)


def _hipcc():
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    h = os.path.join(rocm, "bin", "hipcc")
    return h if os.path.exists(h) else shutil.which("hipcc")


def _newest_header():
    hs = glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True)
    return max((os.path.getmtime(h) for h in hs), default=0.0)


def _compile(cmd, src, obj, verbose):
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed for {src}:\n{r.stdout}\n{r.stderr}")
    return obj


def build(jobs: int | None = None, force: bool = False, verbose: bool = False, out: str | None = None,
          per_file_flags: bool = True) -> str:
    """Compile + link; `out` / `per_file_flags=False` build an A/B variant (own object dir)."""
    OUT_ = out or OUT
    BUILD_ = BUILD if out is None else os.path.join(ROOT, "build", "obj_" + os.path.basename(out).replace(".so", ""))
    tdir, incs, abi = _torch_paths()
    hipcc = _hipcc()
    if hipcc is None:
        raise RuntimeError("hipcc not found (set ROCM_PATH)")
    os.makedirs(BUILD_, exist_ok=True)
    common = [
        "-O3", "-std=c++17", "-fPIC", "-DUSE_ROCM=1", f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
        "-DTORCH_EXTENSION_NAME=_C", "-Wno-unused-result", "-Wno-deprecated-declarations",
    ] + [f"-I{i}" for i in incs] + [f"-I{CSRC}", f"-I{sysconfig.get_paths()['include']}"]
    hip_flags = common + [f"--offload-arch={ARCH}", "-fno-gpu-rdc", "-munsafe-fp-atomics"]
    hip_flags += os.environ.get("DTG_EXTRA_HIPFLAGS", "").split()  # A/B variant builds (with --out)
    cpu_flags = common + ["-march=x86-64-v3", "-fopenmp", "-x", "c++"]
    # Per-file codegen options.  flash_attn.hip: MFMA results in ArchVGPRs.  Its backward kernels
    # keep 128 f32 dK/dV (or dQ) accumulators live across the loop; in the default AGPR form the
    # allocator placed the S / dP tiles in the same AGPRs and copied 32-64 accumulator registers
    # out and back (v_accvgpr_read/write) every item -- 96-128 extra VALU per 32-96 MFMAs in
    # the loop (ISA counted with llvm-objdump).  The VGPR form removes all of them, no spills.
    per_file = {"flash_attn.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form=1"]} if per_file_flags else {}
    srcs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")) + glob.glob(os.path.join(CSRC, "comm", "*.hip")))
    cpu_srcs = sorted(glob.glob(os.path.join(CSRC, "cpu", "*.cpp")))
    hdr_t = _newest_header()
    jobs_list = []
    objs = []
    for src, flags in [(s, hip_flags) for s in srcs] + [(s, cpu_flags) for s in cpu_srcs]:
        rel = os.path.relpath(src, CSRC).replace(os.sep, "_")
        obj = os.path.join(BUILD_, rel + ".o")
        objs.append(obj)
        stale = force or not os.path.exists(obj) or os.path.getmtime(obj) < max(os.path.getmtime(src), hdr_t)
        if stale:
            extra = per_file.get(os.path.basename(src), [])
            jobs_list.append(([hipcc] + flags + extra + ["-c", src, "-o", obj], src, obj))
    jobs = jobs or min(8, os.cpu_count() or 4)
    if jobs_list:
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            futs = [ex.submit(_compile, c, s, o, verbose) for c, s, o in jobs_list]
            for f in cf.as_completed(futs):
                f.result()
    need_link = force or bool(jobs_list) or not os.path.exists(OUT_) or os.path.getmtime(OUT_) < max(os.path.getmtime(o) for o in objs)
    if need_link:
        lib = os.path.join(tdir, "lib")
        link = [hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-fopenmp", "-o", OUT_ + ".tmp"] + objs + [
            f"-L{lib}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", f"-Wl,-rpath,{lib}",
        ]
        _compile(link, "link", OUT_, verbose)
        os.replace(OUT_ + ".tmp", OUT_)
    return OUT_


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", type=int, default=None)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--out", default=None, help="A/B variant: link to this path (objects in build/obj_<name>)")
    ap.add_argument("--no-per-file-flags", action="store_true")
    a = ap.parse_args()
    print(build(a.j, a.force, a.verbose, a.out, not a.no_per_file_flags))
    sys.exit(0)
