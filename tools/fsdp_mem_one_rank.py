#!/usr/bin/env python3
"""Memory of ONE rank of a W-rank FSDP job, measured on one GPU.

A rank's allocations depend on W only through the shard sizes and the gathered units, never on
the values the collectives move.  So this tool runs rank 0 of a W-rank FULL_SHARD job alone,
with PyTorch's `fake` process group standing in for the other W - 1 ranks (every collective
returns at once and leaves its output untouched): the same engine, the same unit layout, the
same allocations and frees in the same order as on a real W-GPU node -- and garbage numerics,
which this tool never reports.  It fills the reference's W = 8 memory row
(`/root/reference/04-fully-sharded-data-parallel/README.md:271-333`) with a measurement instead
of the planner's prediction, and is checked against the real multi-rank runs at W = 1, 2, 4
(`profiles/r2/fsdp_memory_and_host_adamw.md`, `profiles/r3/s07/`).

    python tools/fsdp_mem_one_rank.py --world 8 [--model llama-2-7b --batch 10 --seq 1024]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--model", default="llama-2-7b")
    ap.add_argument("--batch", type=int, default=10)
    ap.add_argument("--seq", type=int, default=1024)
    ap.add_argument("--numel-to-wrap", type=int, default=100_000_000)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--cpu-offload", action="store_true")
    a = ap.parse_args()

    import torch
    import torch.distributed as dist
    from torch.testing._internal.distributed.fake_pg import FakeStore

    import dtg  # noqa: F401
    from dtg.models import build_model, resolve_config
    from dtg.parallel.data_parallel import FlatAdamW
    from dtg.parallel.fsdp import FullyShard

    cuda = torch.cuda.is_available()
    device = torch.device("cuda:0" if cuda else "cpu")
    if cuda:
        torch.cuda.set_device(device)
    dist.init_process_group("fake", store=FakeStore(), rank=0, world_size=a.world)
    cfg = resolve_config(a.model)
    with torch.device("meta"):
        model = build_model(cfg, init=False)
    kw = {"cpu_offload": True} if a.cpu_offload else {}
    engine = FullyShard(model, policy="size", min_num_params=a.numel_to_wrap, device=device, **kw)
    opt = FlatAdamW(engine, lr=3e-5)
    ids = torch.randint(0, cfg.vocab_size, (a.batch, a.seq), device=device)
    gb = 2**30
    valley = peak = 0.0
    t0 = time.perf_counter()
    for _ in range(a.steps):
        if cuda:
            torch.cuda.synchronize()
            torch.cuda.reset_peak_memory_stats(device)
        out = model(input_ids=ids, labels=ids, num_valid=a.batch * (a.seq - 1))
        engine.backward(out.loss)
        opt.step()
        opt.zero_grad()
        del out
        if cuda:
            torch.cuda.synchronize()
            peak = torch.cuda.max_memory_allocated(device) / gb
            valley = torch.cuda.memory_allocated(device) / gb
    rec = {"what": "one rank of a W-rank FSDP FULL_SHARD job, other ranks = fake process group "
                   "(allocations exact, numerics not meaningful)",
           "model": cfg.hf_name or a.model, "world": a.world, "batch_per_gpu": a.batch, "seq_len": a.seq,
           "wrap": f"size>={a.numel_to_wrap}", "cpu_offload": a.cpu_offload, "device": str(device),
           "valley_gib": round(valley, 2), "peak_gib": round(peak, 2),
           "ms_per_step_no_comm": round(1000 * (time.perf_counter() - t0) / max(1, a.steps), 1),
           "shard_params": sum(u.shard_numel for u in engine.units) + (engine.root.shard_numel if engine.root else 0)}
    print(json.dumps(rec), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
