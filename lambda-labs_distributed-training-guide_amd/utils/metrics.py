"""Metric records and sinks.

Keys match the reference (`global_step, lr, running_loss, epoch, epoch_progress,
num_batches_remaining, <mem>, tok/s, time/total, time/{data,forward,backward,update}`); this
framework adds `tok/s/gpu` and `mfu`.  Sinks: the logger (every rank), a JSONL file in the
experiment directory, and wandb on rank 0 when it is installed (it is optional: the GPU boxes
have no network, so `WANDB_MODE=offline` is implied there).
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


class MetricSink:
    def __init__(self, exp_dir, rank: int, use_wandb: bool = True, wandb_kwargs=None):
        self.rank = rank
        self.path = Path(exp_dir) / (f"metrics-rank{rank}.jsonl")
        self.wandb = None
        if use_wandb and rank == 0 and os.environ.get("DTG_NO_WANDB", "0") != "1":
            try:
                import wandb  # noqa: F401

                os.environ.setdefault("WANDB_MODE", "offline")
                self.wandb = wandb
                wandb.init(**(wandb_kwargs or {}))
            except Exception:
                self.wandb = None

    def log(self, info: dict, step: int):
        with open(self.path, "a") as fp:
            fp.write(json.dumps({k: (float(v) if isinstance(v, (int, float)) else v) for k, v in info.items()}) + "\n")
        if self.wandb is not None:
            self.wandb.log(info, step=step)
