"""Debug: the bench_hipgraph GPT-2 setting (cosine schedule, 4 cycled batches, 35 steps), losses per step."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import torch

import dtg  # noqa: F401
from dtg.models import build_model
from dtg.parallel.data_parallel import DataParallel, FlatAdamW
from dtg.train.graph import GraphedStep


def run(graph, sched_on, B=1, S=1024, steps=35):
    dev = torch.device("cuda")
    torch.manual_seed(0)
    m = build_model("gpt2", device=dev)
    m.eval()
    eng = DataParallel(m, mode="single")
    opt = FlatAdamW(eng, lr=3e-5)
    sched = torch.optim.lr_scheduler.CosineAnnealingLR(opt, T_max=1000, eta_min=3e-7) if sched_on else None
    bs = [torch.randint(0, 50257, (B, S), device=dev) for _ in range(4)]
    out = []
    gs = GraphedStep(m, eng, opt, sched, warmup=3, num_valid=B * (S - 1)) if graph else None
    for i in range(steps):
        b = bs[i % 4]
        if graph:
            out.append(gs({"input_ids": b, "labels": b}).item())
        else:
            opt.zero_grad()
            o = m(input_ids=b, labels=b, num_valid=B * (S - 1))
            eng.backward(o.loss)
            opt.step()
            if sched:
                sched.step()
            out.append(o.loss.item())
    return out


for sched_on in (False, True):
    print("sched", sched_on, "eager", [round(x, 3) for x in run(False, sched_on)], flush=True)
    print("sched", sched_on, "graph", [round(x, 3) for x in run(True, sched_on)], flush=True)
