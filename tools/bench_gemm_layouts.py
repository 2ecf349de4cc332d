#!/usr/bin/env python3
"""Time the Llama decoder GEMMs in every operand layout hipBLASLt can be handed.

A Linear layer's three GEMMs see different operand layouts: forward y = x w^T has both
operands K-contiguous ("TN" in BLAS terms), dX = dY w has one K-strided operand ("NN") and
dW = dY^T x has both K-strided ("NT").  MFMA tiles want K-contiguous operands, so this tool
measures what each layout costs and what an explicit transpose (or a transposed weight copy)
would buy back.  Prints one JSON line per (shape, variant).

    python tools/bench_gemm_layouts.py --tokens 16384 [--blas hipblaslt|rocblas]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def shapes(h, i, nh, nkv):
    hd = h // nh
    return {"qkv": ((nh + 2 * nkv) * hd, h), "o": (h, h), "gate_up": (2 * i, h), "down": (h, i)}


def timeit(fn, iters=20):
    import torch

    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=16384)
    ap.add_argument("--blas", default="hipblaslt", choices=["hipblaslt", "rocblas"])
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    import torch

    import dtg.ops  # noqa: F401  (loads the HIP transpose kernel)

    torch.backends.cuda.preferred_blas_library({"rocblas": "cublas", "hipblaslt": "cublaslt"}[a.blas])
    dev = torch.device("cuda")
    T = a.tokens
    for name, (n_out, n_in) in shapes(4096, 14336, 32, 8).items():
        x = torch.randn(T, n_in, device=dev, dtype=torch.bfloat16)
        w = torch.randn(n_out, n_in, device=dev, dtype=torch.bfloat16) * 0.02
        wt = w.t().contiguous()
        dy = torch.randn(T, n_out, device=dev, dtype=torch.bfloat16)
        dyt = dy.t().contiguous()
        xt = x.t().contiguous()
        g = torch.empty(n_out, n_in, device=dev, dtype=torch.bfloat16)
        gt = torch.empty(n_in, n_out, device=dev, dtype=torch.bfloat16)
        yo = torch.empty(T, n_out, device=dev, dtype=torch.bfloat16)
        xo = torch.empty(T, n_in, device=dev, dtype=torch.bfloat16)
        flop = 2.0 * T * n_out * n_in
        variants = {
            "fwd_TN": lambda: torch.mm(x, w.t(), out=yo),
            "dx_NN": lambda: torch.mm(dy, w, out=xo),
            "dx_TN_wT": lambda: torch.mm(dy, wt.t(), out=xo),
            "dw_NT": lambda: torch.mm(dy.t(), x, out=g),
            "dw_NT_swapped": lambda: torch.mm(x.t(), dy, out=gt),
            "dw_TN_pretransposed": lambda: torch.mm(dyt, xt.t(), out=g),
            "transpose_dy": lambda: dyt.copy_(dy.t()),
            "transpose_x": lambda: xt.copy_(x.t()),
            "transpose_dy_hip": lambda: torch.ops.dtg.transpose2d(dy),
            "transpose_x_hip": lambda: torch.ops.dtg.transpose2d(x),
            "transpose_w_hip": lambda: torch.ops.dtg.transpose2d(w),
        }
        for v, fn in variants.items():
            ms = timeit(fn, a.iters)
            rec = {"shape": name, "T": T, "out": n_out, "in": n_in, "variant": v, "blas": a.blas, "ms": round(ms, 4)}
            if v.startswith("transpose"):
                nbytes = 2 * 2 * {"dy": dy, "x": x, "w": w}[v.split("_")[1]].numel()
                rec["GBps"] = round(nbytes / ms / 1e6, 1)
            else:
                rec["TFLOPs"] = round(flop / ms / 1e9, 1)
            print(json.dumps(rec), flush=True)
        del x, w, wt, dy, dyt, xt, g, gt, yo, xo
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
