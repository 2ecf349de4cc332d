#!/usr/bin/env python3
"""The MLP backward's dX GEMM, dX = dGU @ W_gu, at the 8B step shape (T 16384, 2I 28672, H 4096),
timed with the gate/up gradient in the two layouts swiglu_bwd_t can hand it: row-major dGU
[T, 2I] (K-contiguous, the current "TN" call) vs the transposed dGU^T [2I, T] that the weight-
gradient GEMM already needs (M-contiguous A) -- if the second is as fast, the kernel need not
write dGU at all (0.94 GB per layer).  Median of interleaved rounds, TF/s."""
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402


def main():
    T, K, N = 16384, 28672, 4096
    dev = torch.device("cuda:0")
    dgu = torch.randn(T, K, device=dev).bfloat16()
    dguT = dgu.t().contiguous()
    wT = torch.randn(N, K, device=dev).bfloat16()  # W_gu^T as the engine keeps it ([H, 2I])
    w = wT.t().contiguous()                          # W_gu [2I, H]
    variants = {
        "tn_rowmajor_dgu": lambda: torch.mm(dgu, wT.t()),
        "nn_transposed_dgu": lambda: torch.mm(dguT.t(), wT.t()),
        "nn_transposed_dgu_w": lambda: torch.mm(dguT.t(), w),
    }
    ref = variants["tn_rowmajor_dgu"]().float()
    for k, f in variants.items():
        err = ((f().float() - ref).norm() / ref.norm()).item()
        print(k, "rel err vs TN", err, flush=True)
    times = {k: [] for k in variants}
    for _ in range(7):
        for k, f in variants.items():
            for _ in range(3):
                f()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                f()
            e1.record()
            torch.cuda.synchronize()
            times[k].append(e0.elapsed_time(e1) / 10)
    for k, v in times.items():
        ms = statistics.median(v)
        print({"variant": k, "ms": round(ms, 3), "TFLOPs": round(2 * T * K * N / ms / 1e9, 1)}, flush=True)


if __name__ == "__main__":
    main()
