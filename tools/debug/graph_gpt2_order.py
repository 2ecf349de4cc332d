"""Debug: GPT-2 graph replays with the batch order of bench_hipgraph (0,1,2,3,0 | 0,1,2)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import torch

import dtg  # noqa: F401
from dtg.models import build_model
from dtg.parallel.data_parallel import DataParallel, FlatAdamW
from dtg.train.graph import GraphedStep


def run(order, sync, graph=True):
    dev = torch.device("cuda")
    torch.manual_seed(0)
    model = build_model("gpt2", device=dev)
    model.eval()
    eng = DataParallel(model, mode="single")
    opt = FlatAdamW(eng, lr=3e-5)
    sched = torch.optim.lr_scheduler.CosineAnnealingLR(opt, T_max=1000, eta_min=3e-7)
    B, S = 1, 1024
    batches = [torch.randint(0, 50257, (B, S), device=dev) for _ in range(4)]
    gs = GraphedStep(model, eng, opt, sched, warmup=3, num_valid=B * (S - 1))
    out = []
    for j, i in enumerate(order):
        loss = gs({"input_ids": batches[i], "labels": batches[i]})
        if sync:
            torch.cuda.synchronize()
            out.append(round(loss.item(), 4))
    torch.cuda.synchronize()
    bad = [n for n, p in model.named_parameters() if not torch.isfinite(p).all()]
    return out, loss.item(), bad[:2]


print("bench order, sync  ", run([0, 1, 2, 3, 0, 0, 1, 2], True), flush=True)
print("bench order, nosync", run([0, 1, 2, 3, 0, 0, 1, 2], False), flush=True)
print("cyclic order, nosync", run([0, 1, 2, 3, 0, 1, 2, 3], False), flush=True)
print("sync after 5, then nosync", run([0, 1, 2, 3, 0], True), flush=True)
