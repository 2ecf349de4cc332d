#!/usr/bin/env python3
"""Eager vs HIP-graph-replayed training step (dtg.train.graph.GraphedStep) for launch-bound
configurations: GPT-2 124M (the reference's chapter 01/02 default model) and small Llama
shapes at small batch.  Prints one JSON line per (model, batch, mode).

    python tools/bench_hipgraph.py --models gpt2,llama-tiny-d128 --batches 1,8 --seq 1024
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def run(name, B, S, steps, graph, dropout, torch):
    from dtg.models import build_model
    from dtg.parallel.data_parallel import DataParallel, FlatAdamW
    from dtg.train.graph import GraphedStep

    dev = torch.device("cuda")
    torch.manual_seed(0)
    model = build_model(name, device=dev)
    if not dropout:
        model.eval()
    eng = DataParallel(model, mode="single")
    opt = FlatAdamW(eng, lr=3e-5)
    sched = torch.optim.lr_scheduler.CosineAnnealingLR(opt, T_max=1000, eta_min=3e-7)
    V = model.config.vocab_size
    batches = [torch.randint(0, V, (B, S), device=dev) for _ in range(4)]
    nv = B * (S - 1)
    if graph:
        gs = GraphedStep(model, eng, opt, sched, warmup=3, num_valid=nv)
        step = lambda b: gs({"input_ids": b, "labels": b})
    else:
        def step(b):
            opt.zero_grad()
            out = model(input_ids=b, labels=b, num_valid=nv)
            eng.backward(out.loss)
            opt.step()
            sched.step()
            return out.loss
    for i in range(5):
        l0 = step(batches[i % 4])
        if os.environ.get("DTG_HIPGRAPH_CHECK"):
            torch.cuda.synchronize()
            bad = [n for n, p in model.named_parameters() if not torch.isfinite(p).all()]
            print(f"[check] {name} graph={graph} warm step {i}: loss {l0.item():.4f} bad {bad[:3]}", file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        loss = step(batches[i % 4])
    torch.cuda.synchronize()
    ms = 1000 * (time.perf_counter() - t0) / steps
    bad = [n for n, p in model.named_parameters() if not torch.isfinite(p).all()]
    if bad:
        print(f"[bench_hipgraph] non-finite parameters after {name} {'graph' if graph else 'eager'}: {bad[:4]}",
              file=sys.stderr, flush=True)
    return {"model": name, "batch": B, "seq": S, "mode": "hipgraph" if graph else "eager", "dropout": dropout,
            "ms_per_step": round(ms, 3), "tok_per_s": round(B * S / ms * 1000, 1), "loss": round(float(loss.item()), 4)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default="gpt2,llama-tiny-d128")
    ap.add_argument("--batches", default="1,8")
    ap.add_argument("--seq", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--dropout", action="store_true", help="train mode (GPT-2 dropout 0.1) instead of eval-mode dropout-free")
    ap.add_argument("--modes", default="eager,hipgraph")
    a = ap.parse_args()
    import torch

    import dtg  # noqa: F401

    for name in a.models.split(","):
        for B in [int(x) for x in a.batches.split(",")]:
            for graph in [m == "hipgraph" for m in a.modes.split(",")]:
                print(json.dumps(run(name, B, a.seq, a.steps, graph, a.dropout, torch)), flush=True)
                torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
