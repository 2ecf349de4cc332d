#!/usr/bin/env python3
"""The hand-written token-major weight-gradient GEMM (csrc/kernels/dw_gemm.hip) against what the
Linear backward runs today, on the Llama-3-8B decoder's dW shapes.

Variants per shape (dW = dY^T X, dY [T, out], X [T, in], bf16, f32 accumulation):
  * hand          dtg::dw_gemm_ on the token-major operands as they are (no transposes),
                  k-step pipeline (variant 2); hand_v1 the K-tile pipeline (variant 1); hand_v3
                  the k-step pipeline with the 8-phase template's wave-group ping-pong; hand_v4
                  the k-step pipeline on a 10-slot LDS ring, 8 quarters in flight; hand_v5 the
                  same ring with 2 k-steps per barrier, 6 quarters in flight (variants 6-9 were
                  measured in profiles/r4/s16, s20 and removed);
  * hand_acc      the same, accumulating into the gradient (addmm_ semantics);
  * tn_gemm       hipBLASLt on pre-transposed, K-contiguous operands (the GEMM alone);
  * tn_total      transpose dY + transpose X + tn_gemm (what the default backward pays);
  * nt            hipBLASLt handed the strided layout directly (no transposes).
The same TunableOp table as bench.py is used for hipBLASLt.  Prints one JSON line per row and
the hand kernel's max relative error against an f32 product.

    python tools/bench_dw_gemm.py [--tokens 16384] [--iters 20]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def shapes(h=4096, i=14336, nh=32, nkv=8):
    hd = h // nh
    return {"qkv": ((nh + 2 * nkv) * hd, h), "o": (h, h), "gate_up": (2 * i, h), "down": (h, i)}


def timeit(fn, iters):
    import torch

    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        ts.append((s, e))
    torch.cuda.synchronize()
    ms = sorted(s.elapsed_time(e) for s, e in ts)
    return ms[len(ms) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=16384)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--tunableop", choices=["off", "use"], default="use")
    ap.add_argument("--only", default=None, help="comma list of shape names")
    a = ap.parse_args()
    import torch

    import dtg.ops  # noqa: F401

    if a.tunableop == "use":
        from dtg.utils.gemm_tuning import enable_tunableop

        enable_tunableop(tune=False)
    dev = torch.device("cuda")
    T = a.tokens
    g = torch.Generator(device=dev).manual_seed(0)
    tot = {}
    for name, (n_out, n_in) in shapes().items():
        if a.only and name not in a.only.split(","):
            continue
        dy = torch.randn(T, n_out, device=dev, dtype=torch.bfloat16, generator=g)
        x = torch.randn(T, n_in, device=dev, dtype=torch.bfloat16, generator=g)
        dyt, xt = dy.t().contiguous(), x.t().contiguous()
        out = torch.empty(n_out, n_in, device=dev, dtype=torch.bfloat16)
        ref = dy.float().t() @ x.float()
        errs = {}
        for v in ("1", "2", "3", "4", "5"):
            os.environ["DTG_DWG_VARIANT"] = v
            out.fill_(float("nan"))
            torch.ops.dtg.dw_gemm_(dy, x, out, False)
            errs[v] = ((out.float() - ref).abs().max() / ref.abs().max()).item()
        err = max(errs.values())
        out2 = out.clone()
        torch.ops.dtg.dw_gemm_(dy, x, out2, True)
        err_acc = ((out2.float() - 2 * ref).abs().max() / (2 * ref).abs().max()).item()
        del ref
        flop = 2.0 * T * n_out * n_in
        def hand(v, acc=False):
            def fn():
                os.environ["DTG_DWG_VARIANT"] = v
                torch.ops.dtg.dw_gemm_(dy, x, out, acc)
            return fn

        variants = {
            "hand": hand("2"),
            "hand_v1": hand("1"),
            "hand_v3": hand("3"),
            "hand_v4": hand("4"),
            "hand_v5": hand("5"),
            "hand_acc": hand("2", True),
            "tn_gemm": lambda: torch.mm(dyt, xt.t(), out=out),
            "tn_total": lambda: torch.mm(torch.ops.dtg.transpose2d(dy), torch.ops.dtg.transpose2d(x).t(), out=out),
            "nt": lambda: torch.mm(dy.t(), x, out=out),
        }
        for v, fn in variants.items():
            ms = timeit(fn, a.iters)
            tot[v] = tot.get(v, 0.0) + ms
            rec = {"shape": name, "T": T, "out": n_out, "in": n_in, "variant": v, "ms": round(ms, 4),
                   "TFLOPs": round(flop / ms / 1e9, 1)}
            if v == "hand":
                rec["max_rel_err"] = err
                rec["max_rel_err_acc"] = err_acc
            print(json.dumps(rec), flush=True)
        del dy, x, dyt, xt, out, out2
        torch.cuda.empty_cache()
    print(json.dumps({"per_layer_ms": {k: round(v, 4) for k, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
