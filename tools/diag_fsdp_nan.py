#!/usr/bin/env python3
"""Localise a NaN seen in tests/test_xgmi_dp_gpu.py's FSDP reference run (world 1): train the
test's 6-layer tiny Llama with FullyShard at 8 and 16 rows per step (two micro-batches) and with
DataParallel, print per-step losses and which parameters go non-finite."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

import dtg  # noqa: E402,F401


def run(engine_kind, rows, layers=6, steps=3):
    from dtg.models import build_model, resolve_config
    from dtg.parallel.data_parallel import DataParallel, FlatAdamW
    from dtg.parallel.fsdp import FullyShard

    dev = torch.device("cuda:0")
    cfg = resolve_config("llama-tiny-d128", num_hidden_layers=layers)
    torch.manual_seed(0)
    model = build_model(cfg, device=dev)
    eng = FullyShard(model, device=dev) if engine_kind == "fsdp" else DataParallel(model, mode="single")
    opt = FlatAdamW(eng, lr=1e-3)
    g = torch.Generator().manual_seed(0)
    out_rec = []
    for _ in range(steps):
        ids = torch.randint(0, cfg.vocab_size, (rows, 128), generator=g).to(dev)
        opt.zero_grad()
        for j, mb in enumerate(ids.chunk(2)):
            ctx = eng.no_sync() if j == 0 else torch.enable_grad()
            with ctx:
                o = model(input_ids=mb, labels=mb)
                eng.backward(o.loss)
        opt.step()
        out_rec.append(round(o.loss.item(), 5))
    torch.cuda.synchronize()
    if engine_kind == "fsdp":
        sd = eng.full_state_dict(rank0_only=False)
    else:
        sd = {n: p.detach() for n, p in model.named_parameters()}
    bad = [k for k, v in sd.items() if not torch.isfinite(v.float()).all()]
    print(engine_kind, rows, "losses", out_rec, "non-finite params:", len(bad), bad[:6], flush=True)


if __name__ == "__main__":
    for kind in ("single", "fsdp"):
        for rows in (8, 16):
            run(kind, rows)
