#!/usr/bin/env python3
"""Diagnostic: W^T engine vs plain engine on the GPU, per-parameter max |diff| / count after 3
steps.  Variants: plain, plain again (run-to-run control), weight_t, weight_t with the copies
never used (isolates the optimizer kernel from the dX GEMM operand source)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

import dtg  # noqa: E402,F401
from dtg.models import build_model, resolve_config  # noqa: E402
from dtg.parallel.data_parallel import DataParallel, FlatAdamW  # noqa: E402


def run(variant, cfg, batches, dev):
    torch.manual_seed(0)
    m = build_model(cfg, device=dev)
    eng = DataParallel(m, mode="single", weight_t=variant in ("wt", "wt_unused"))
    if variant == "wt_unused":
        eng.weight_t = lambda i: None
    opt = FlatAdamW(eng, lr=1e-3)
    for ids in batches:
        opt.zero_grad()
        out = m(input_ids=ids, labels=ids)
        eng.backward(out.loss)
        opt.step()
    torch.cuda.synchronize()
    return {n: p.detach().float().clone() for n, p in m.named_parameters()}


def main():
    dev = torch.device("cuda")
    cfg = resolve_config(sys.argv[1] if len(sys.argv) > 1 else "llama-tiny-d128")
    g = torch.Generator().manual_seed(0)
    batches = [torch.randint(0, cfg.vocab_size, (4, 1024), generator=g).to(dev) for _ in range(3)]
    res = {v: run(v, cfg, batches, dev) for v in ("plain", "again", "wt", "wt_unused")}
    for v in ("again", "wt", "wt_unused"):
        bad = [(n, (res[v][n] - t).abs().max().item(), int((res[v][n] != t).sum())) for n, t in res["plain"].items()
               if not torch.equal(res[v][n], t)]
        print(v, "differs in", len(bad), "params:", bad[:8], flush=True)


if __name__ == "__main__":
    main()
