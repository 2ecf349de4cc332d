"""Debug: bench_hipgraph.run() for GPT-2 with per-step finiteness checks."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import torch

import dtg  # noqa: F401
from dtg.models import build_model
from dtg.parallel.data_parallel import DataParallel, FlatAdamW
from dtg.train.graph import GraphedStep


def run(variant):
    dev = torch.device("cuda")
    torch.manual_seed(0)
    model = build_model("gpt2", device=dev)
    model.eval()
    eng = DataParallel(model, mode="single")
    opt = FlatAdamW(eng, lr=3e-5)
    sched = torch.optim.lr_scheduler.CosineAnnealingLR(opt, T_max=1000, eta_min=3e-7)
    B, S = 1, 1024
    if variant == "bs_before_gs":
        batches = [torch.randint(0, 50257, (B, S), device=dev) for _ in range(4)]
        gs = GraphedStep(model, eng, opt, sched, warmup=3, num_valid=B * (S - 1))
    else:
        gs = GraphedStep(model, eng, opt, sched, warmup=3, num_valid=B * (S - 1))
        batches = [torch.randint(0, 50257, (B, S), device=dev) for _ in range(4)]
    for i in range(10):
        loss = gs({"input_ids": batches[i % 4], "labels": batches[i % 4]})
        if variant != "nosync":
            torch.cuda.synchronize()
            bad = [n for n, p in model.named_parameters() if not torch.isfinite(p).all()]
            gbad = [n for n, p in model.named_parameters() if not torch.isfinite(p.main_grad).all()]
            print(variant, i, round(loss.item(), 4), "bad params", bad[:3], "bad grads", gbad[:3], flush=True)
    torch.cuda.synchronize()
    print(variant, "final", loss.item(), flush=True)


for v in ("bs_before_gs", "gs_before_bs", "nosync"):
    run(v)
