"""Debug: eager vs HIP-graph losses per step for GPT-2 variants (finds where replays diverge)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import torch

import dtg  # noqa: F401
from dtg.models import build_model, resolve_config
from dtg.parallel.data_parallel import DataParallel, FlatAdamW
from dtg.train.graph import GraphedStep


def run(cfg, graph, B=1, S=1024, steps=8):
    dev = torch.device("cuda")
    torch.manual_seed(0)
    m = build_model(cfg, device=dev)
    m.eval()
    eng = DataParallel(m, mode="single")
    opt = FlatAdamW(eng, lr=3e-5)
    g = torch.Generator(device=dev).manual_seed(5)
    bs = [torch.randint(0, cfg.vocab_size, (B, S), device=dev, generator=g) for _ in range(steps)]
    out = []
    if graph:
        gs = GraphedStep(m, eng, opt, None, warmup=2, num_valid=B * (S - 1))
        for b in bs:
            out.append(gs({"input_ids": b, "labels": b}).item())
    else:
        for b in bs:
            opt.zero_grad()
            o = m(input_ids=b, labels=b, num_valid=B * (S - 1))
            eng.backward(o.loss)
            opt.step()
            out.append(o.loss.item())
    return out


for name, over in [("gpt2", {}), ("gpt2", {"n_layer": 2}), ("gpt2", {"vocab_size": 50304}),
                   ("gpt2", {"n_layer": 2, "vocab_size": 50304}), ("gpt2-tiny", {"n_positions": 1024})]:
    cfg = resolve_config(name, **over)
    e = run(cfg, False)
    gr = run(cfg, True)
    print(name, over, "eager", [round(x, 4) for x in e], flush=True)
    print(name, over, "graph", [round(x, 4) for x in gr], flush=True)
