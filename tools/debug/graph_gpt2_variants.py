"""Debug: which change removes the GPT-2 replay NaN seen in tools/bench_hipgraph.py."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch

import dtg  # noqa: F401
import bench_hipgraph as bh
from dtg.train import graph as G

orig_write = G.GraphedStep._write_hyper


def blocking_write(self):
    g = self.opt.param_groups[0]
    t = self.engine.step_count + 1
    b1, b2 = g["betas"]
    import math
    self._hyper.copy_(torch.tensor([g["lr"], 1.0 - b1 ** t, math.sqrt(1.0 - b2 ** t)], dtype=torch.float32))


for variant in ("baseline", "blocking_hyper", "baseline_again"):
    G.GraphedStep._write_hyper = blocking_write if variant == "blocking_hyper" else orig_write
    r = bh.run("gpt2", 1, 1024, 3, True, False, torch)
    print(variant, r["loss"], flush=True)
    torch.cuda.empty_cache()
