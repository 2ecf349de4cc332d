#!/usr/bin/env python3
"""Tune the hipBLASLt/rocBLAS solution of every Linear GEMM of a model with PyTorch TunableOp,
one shape at a time, and merge the winners into the committed table (tunableop/).

Each GEMM is issued exactly as the training step issues it (ops.functional._Linear: forward
x @ w^T, dX = dY @ w, dW = dY^T @ x into a preallocated gradient), so the TunableOp keys match.
A heartbeat line is printed every 30 s while a shape is being tuned.

    python tools/tune_gemms.py --model llama-3-8b --tokens 16384 --which dw
"""
import argparse
import os
import sys
import threading
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def shapes(cfg):
    h, i = cfg.hidden_size, cfg.intermediate_size
    hd = h // cfg.num_attention_heads
    qkv = (cfg.num_attention_heads + 2 * cfg.num_key_value_heads) * hd
    return {"qkv": (qkv, h), "o": (h, h), "gate_up": (2 * i, h), "down": (h, i), "lm_head": (cfg.vocab_size, h)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--tokens", type=int, default=16384)
    ap.add_argument("--which", default="dw", help="comma list of fwd,dx,dw,dx_tn,dw_tn")
    ap.add_argument("--only", default="", help="comma list of qkv,o,gate_up,down")
    ap.add_argument("--out", default="gpurun_out/tunableop_new.csv")
    ap.add_argument("--max-ms", type=int, default=20)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    import torch

    import dtg  # noqa: F401
    from dtg.models import resolve_config

    cfg = resolve_config(a.model)
    t = torch.cuda.tunable
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    t.enable(True)
    t.set_filename(a.out, insert_device_ordinal=False)
    t.tuning_enable(True)
    t.set_max_tuning_duration(a.max_ms)
    t.set_max_tuning_iterations(a.iters)
    current = {"name": "", "t0": time.time()}

    def beat():
        while True:
            time.sleep(30)
            print(f"[tune] {current['name']} ... {time.time() - current['t0']:.0f}s", flush=True)

    threading.Thread(target=beat, daemon=True).start()
    dev = torch.device("cuda")
    T = a.tokens
    which = a.which.split(",")
    only = [s for s in a.only.split(",") if s]
    for name, (out_f, in_f) in shapes(cfg).items():
        if (only and name not in only) or (not only and name == "lm_head"):
            continue  # the loss head runs per chunk: tune it with --only lm_head --tokens <chunk>
        x = torch.randn(T, in_f, device=dev, dtype=torch.bfloat16)
        w = torch.randn(out_f, in_f, device=dev, dtype=torch.bfloat16) * 0.02
        dy = torch.randn(T, out_f, device=dev, dtype=torch.bfloat16)
        mg = torch.empty(out_f, in_f, device=dev, dtype=torch.bfloat16)
        wt, dyt, xt = w.t().contiguous(), dy.t().contiguous(), x.t().contiguous()
        jobs = {"fwd": lambda: torch.mm(x, w.t()), "dx": lambda: torch.mm(dy, w),
                "dw": lambda: torch.mm(dy.t(), x, out=mg),
                # the TN forms issued by ops.functional._Linear (DTG_LINEAR_BWD=tn, the default)
                "dx_tn": lambda: torch.mm(dy, wt.t()), "dw_tn": lambda: torch.mm(dyt, xt.t(), out=mg)}
        for k in which:
            current["name"], current["t0"] = f"{name}/{k}", time.time()
            jobs[k]()
            torch.cuda.synchronize()
            print(f"[tune] {name}/{k} done in {time.time() - current['t0']:.1f}s", flush=True)
        del x, w, dy, mg, wt, dyt, xt
        torch.cuda.empty_cache()
    from dtg.utils.gemm_tuning import save_tunableop

    save_tunableop(a.out)
    print(f"[tune] wrote {a.out}", flush=True)


if __name__ == "__main__":
    main()
