"""Debug: GPT-2 graph replays with and without a host sync per step (host run-ahead)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import torch

import dtg  # noqa: F401
from dtg.models import build_model
from dtg.parallel.data_parallel import DataParallel, FlatAdamW
from dtg.train.graph import GraphedStep


def run(sync_each, B=1, S=1024, steps=35, empty=False):
    dev = torch.device("cuda")
    torch.manual_seed(0)
    m = build_model("gpt2", device=dev)
    m.eval()
    eng = DataParallel(m, mode="single")
    opt = FlatAdamW(eng, lr=3e-5)
    sched = torch.optim.lr_scheduler.CosineAnnealingLR(opt, T_max=1000, eta_min=3e-7)
    bs = [torch.randint(0, 50257, (B, S), device=dev) for _ in range(4)]
    gs = GraphedStep(m, eng, opt, sched, warmup=3, num_valid=B * (S - 1))
    trace = []
    for i in range(steps):
        loss = gs({"input_ids": bs[i % 4], "labels": bs[i % 4]})
        if sync_each:
            trace.append(round(loss.item(), 3))
    torch.cuda.synchronize()
    nan_params = [n for n, p in m.named_parameters() if not torch.isfinite(p).all()]
    return loss.item(), trace[-3:], nan_params[:5]


print("sync each step:", run(True), flush=True)
print("run ahead     :", run(False), flush=True)
