"""Debug: which tensors turn non-finite after GPT-2 HIP-graph replays (order 0,1,2,3,0,0,1)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import torch

import dtg  # noqa: F401
from dtg.models import build_model
from dtg.parallel.data_parallel import DataParallel, FlatAdamW
from dtg.train.graph import GraphedStep

dev = torch.device("cuda")
torch.manual_seed(0)
model = build_model("gpt2", device=dev)
model.eval()
eng = DataParallel(model, mode="single")
opt = FlatAdamW(eng, lr=3e-5)
B, S = 1, 1024
batches = [torch.randint(0, 50257, (B, S), device=dev) for _ in range(4)]
sched = torch.optim.lr_scheduler.CosineAnnealingLR(opt, T_max=1000, eta_min=3e-7)
gs = GraphedStep(model, eng, opt, sched, warmup=3, num_valid=B * (S - 1))
names = {id(p): n for n, p in model.named_parameters()}
for j, i in enumerate([0, 1, 2, 3, 0, 0, 1]):
    loss = gs({"input_ids": batches[i], "labels": batches[i]})
    torch.cuda.synchronize()
    bp = [n for n, p in model.named_parameters() if not torch.isfinite(p).all()]
    bg = [n for n, p in model.named_parameters() if not torch.isfinite(p.main_grad).all()]
    gmax = max(p.main_grad.float().abs().max().item() for p in model.named_parameters() for p in [p[1]])
    print("   lr", opt.param_groups[0]["lr"], "hyper", gs._hyper.tolist(), "step_count", eng.step_count, flush=True)
    print(j, "batch", i, "loss", round(loss.item(), 4), "graph" if gs.graph is not None else "eager",
          "bad params", bp[:3], "bad grads", bg[:3], "max|g|", gmax,
          "ea", torch.isfinite(eng.exp_avg).all().item(), "eas", torch.isfinite(eng.exp_avg_sq).all().item(), flush=True)
    if bg:
        for n, p in model.named_parameters():
            if n in bg[:3]:
                g = p.main_grad.float()
                print("   ", n, tuple(g.shape), "nonfinite", (~torch.isfinite(g)).sum().item(), flush=True)
