"""Metric records and sinks.

Keys match the reference (`global_step, lr, running_loss, epoch, epoch_progress,
num_batches_remaining, <mem>, tok/s, time/total, time/{data,forward,backward,update}`); this
framework adds `tok/s/gpu` and `mfu`.  Sinks: the logger (every rank), a JSONL file in the
experiment directory, and wandb when it is installed (it is optional: the GPU boxes have no
network, so `WANDB_MODE=offline` is implied there).

wandb run layouts (`--wandb-mode`, reference related-topics/wandb-configurations/README.md):
  rank0        one run from global rank 0: id = name = experiment name, dir = exp_dir
  local_rank0  one run per node (local rank 0 of every node), grouped by the experiment name:
               id = "<experiment>-<rank>", name = "rank-<rank>", dir = exp_dir/rank-<rank>
  every_rank   one run per rank, grouped the same way
All modes pass save_code=True and resume="must" on a resumed experiment.
"""
from __future__ import annotations

import json
import os
from pathlib import Path

import torch

MI355X_BF16_DENSE_FLOPS = 2.5e15


def get_mem_stats(device, suffix: str = "_gb"):
    """Reference `get_mem_stats`: suffix "_gb" (ch01-04,06,07) or "_in_gb" (ch05, deepspeed)."""
    if device.type != "cuda":
        return {}
    free, total = torch.cuda.mem_get_info(device)
    st = torch.cuda.memory_stats(device)
    g = 1e-9
    return {
        f"total{suffix}": g * total,
        f"curr_alloc{suffix}": g * st.get("allocated_bytes.all.current", 0),
        f"peak_alloc{suffix}": g * st.get("allocated_bytes.all.peak", 0),
        f"curr_resv{suffix}": g * st.get("reserved_bytes.all.current", 0),
        f"peak_resv{suffix}": g * st.get("reserved_bytes.all.peak", 0),
    }


WANDB_MODES = ("rank0", "local_rank0", "every_rank")


def wandb_init_kwargs(mode: str, exp_dir, experiment_name: str, rank: int, local_rank: int, resumed: bool,
                      config=None, project: str = "distributed-training-guide"):
    """wandb.init kwargs of this rank for `mode`, or None if this rank does not log to wandb."""
    assert mode in WANDB_MODES, mode
    if mode == "rank0" and rank != 0 or mode == "local_rank0" and local_rank != 0:
        return None
    kw = dict(project=project, resume="must" if resumed else None, save_code=True, config=config)
    if mode == "rank0":
        kw.update(dir=str(exp_dir), id=experiment_name, name=experiment_name)
    else:
        d = Path(exp_dir) / f"rank-{rank}"
        d.mkdir(parents=True, exist_ok=True)
        kw.update(dir=str(d), group=experiment_name, name=f"rank-{rank}", id=f"{experiment_name}-{rank}")
    return kw


class MetricSink:
    def __init__(self, exp_dir, rank: int, use_wandb: bool = True, wandb_kwargs=None):
        """`wandb_kwargs`: this rank's wandb.init kwargs (`wandb_init_kwargs`), None = no wandb
        run on this rank."""
        self.rank = rank
        self.path = Path(exp_dir) / (f"metrics-rank{rank}.jsonl")
        self.wandb = None
        if use_wandb and wandb_kwargs is not None and os.environ.get("DTG_NO_WANDB", "0") != "1":
            try:
                import wandb  # noqa: F401

                os.environ.setdefault("WANDB_MODE", "offline")
                self.wandb = wandb
                wandb.init(**wandb_kwargs)
            except Exception:
                self.wandb = None

    def log(self, info: dict, step: int):
        with open(self.path, "a") as fp:
            fp.write(json.dumps({k: (float(v) if isinstance(v, (int, float)) else v) for k, v in info.items()}) + "\n")
        if self.wandb is not None:
            self.wandb.log(info, step=step)
