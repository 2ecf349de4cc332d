#!/usr/bin/env python3
"""Memory-bound HIP kernels at the Llama-3-8B training shape (16,384 tokens): achieved HBM
bandwidth per kernel from timed launches and the bytes each kernel must move (roofline check
against MI355X's ~6.3 TB/s achievable, 8 TB/s peak).  Pair with `rocprofv3 --pmc FETCH_SIZE`
/ `--pmc WRITE_SIZE` to confirm the byte counts.

    python tools/bench_kernels.py [--tokens 16384]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def timeit(torch, fn, iters=20):
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
    ap.add_argument("--hidden", type=int, default=4096)
    ap.add_argument("--inter", type=int, default=14336)
    ap.add_argument("--params", type=float, default=8.03e9, help="AdamW buffer length")
    ap.add_argument("--layers", type=int, default=8, help="decoder layers of matrices for adamw_t_")
    ap.add_argument("--only", default="", help="run only the cases whose name contains one of these (comma-separated)")
    a = ap.parse_args()
    import torch

    import dtg.ops  # noqa: F401

    ops = torch.ops.dtg
    dev = torch.device("cuda")
    T, H, I = a.tokens, a.hidden, a.inter
    bf = dict(device=dev, dtype=torch.bfloat16)
    x = torch.randn(T, H, **bf)
    res = torch.randn(T, H, **bf)
    w = torch.ones(H, **bf)
    dy = torch.randn(T, H, **bf)
    gu = torch.randn(T, 2 * I, **bf)
    dh = torch.randn(T, I, **bf)
    y, hh, rstd = ops.add_rmsnorm_fwd(x, res, w, 1e-5)
    E = 2  # bytes per bf16
    cases = {
        "add_rmsnorm_fwd": (lambda: ops.add_rmsnorm_fwd(x, res, w, 1e-5), 4 * T * H * E),
        "rmsnorm_bwd(+dres)": (lambda: ops.rmsnorm_bwd(dy, hh, w, rstd, dy), 4 * T * H * E),
        "swiglu_fwd": (lambda: ops.swiglu_fwd(gu), 3 * T * I * E),
    }
    cases["swiglu_bwd_t (dgu, dgu^T, h^T)"] = (lambda: ops.swiglu_bwd_t(dh, gu), (3 + 5) * T * I * E)
    cases["transpose [T,H]"] = (lambda: ops.transpose2d(x), 2 * T * H * E)
    cases["transpose [T,2I]"] = (lambda: ops.transpose2d(gu), 2 * T * 2 * I * E)
    n = int(a.params) // 16 * 16
    n = min(n, 2_000_000_000)  # keep the AdamW buffers at <= 14 GB
    p = torch.randn(n, **bf)
    g = torch.randn(n, **bf)
    m = torch.zeros(n, **bf)
    v = torch.zeros(n, **bf)
    cases["adamw (bf16 p/g/m/v)"] = (lambda: ops.adamw_(p, None, g, m, v, 1e-4, 0.9, 0.999, 1e-8, 0.01, 3, 1.0), 14 * n)
    # adamw_t_ over Llama-3-8B's matrix shapes (a.layers decoder layers), each tile width
    shapes = [(6144, H), (H, H), (2 * I, H), (H, I)] * a.layers
    for tc in (64, 128, 256):
        desc, off, toff, tile0 = [], 0, 0, 0
        for r, c in shapes:
            desc.append([off, r, c, toff, tile0])
            off += r * c
            toff += r * c
            tile0 += -(-r // 64) * -(-c // tc)
        nt = off
        pw, gw = torch.randn(nt, **bf), torch.randn(nt, **bf)
        mw, vw, ptw = torch.zeros(nt, **bf), torch.zeros(nt, **bf), torch.empty(nt, **bf)
        mats = torch.tensor(desc, dtype=torch.long, device=dev)
        runs = {f"adamw_t_ 64x{tc} (+W^T)": (lambda tc=tc, mats=mats, tile0=tile0: ops.adamw_t_(
            pw, None, gw, mw, vw, ptw, mats, tile0, 1e-4, 0.9, 0.999, 1e-8, 0.01, 3, 1.0, None, tc), 16 * nt)}
        if tc == 128:  # the tile walk with no transposed copies (toff = -1): layout effect alone
            mats_nt = mats.clone()
            mats_nt[:, 3] = -1
            runs["adamw_t_ 64x128 tile walk, no W^T"] = (lambda: ops.adamw_t_(
                pw, None, gw, mw, vw, ptw, mats_nt, tile0, 1e-4, 0.9, 0.999, 1e-8, 0.01, 3, 1.0, None, tc), 14 * nt)
            runs["adamw_ (same buffers)"] = (lambda: ops.adamw_(pw, None, gw, mw, vw, 1e-4, 0.9, 0.999, 1e-8, 0.01, 3, 1.0),
                                             14 * nt)
        for name, (fn, nbytes) in runs.items():
            if a.only and not any(o in name for o in a.only.split(',')):
                continue
            ms = timeit(torch, fn)
            print(json.dumps({"kernel": name, "ms": round(ms, 4), "bytes": nbytes, "TBps": round(nbytes / ms / 1e9, 2)}),
                  flush=True)
        del pw, gw, mw, vw, ptw, runs
        torch.cuda.empty_cache()
    for name, (fn, nbytes) in cases.items():
        if a.only and not any(o in name for o in a.only.split(',')):
            continue
        ms = timeit(torch, fn)
        print(json.dumps({"kernel": name, "ms": round(ms, 4), "bytes": nbytes, "TBps": round(nbytes / ms / 1e9, 2)}),
              flush=True)


if __name__ == "__main__":
    main()
