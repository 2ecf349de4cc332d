#!/usr/bin/env python3
"""Headline benchmark: causal-LM pretraining throughput on MI355X (BASELINE.json metric).

    python bench.py --gpus N --steps K --warmup W            (N=1)
    torchrun --nproc-per-node N bench.py --gpus N ...         (N>1, one rank per GPU, RCCL)

Config: Llama-3-8B (bundled config, random init, pure bf16 params/grads/AdamW states as in the
reference), synthetic token data, seq 1024, fixed per-GPU micro-batch (weak scaling). Every
timed step does the full work: forward, backward with overlapped bucketed gradient
reduce-scatter, fused AdamW on the local shard, parameter all-gather and the cosine LR step.
K steps are bracketed by barrier + device synchronize on both sides; the slowest rank's time is
reported.  Rank 0 prints one JSON line (value = whole-job tokens/s).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--batch-size", type=int, default=16, help="per-GPU micro-batch (sequences)")
    ap.add_argument("--seq-len", type=int, default=1024)
    ap.add_argument("--parallel", default="zero", choices=["ddp", "zero", "fsdp"])
    ap.add_argument("--bucket-mb", type=int, default=256)
    ap.add_argument("--overlap-optimizer", type=int, default=0,
                    help="1: per-bucket AdamW (and ZeRO all-gather) on a side stream during backward (measured +0.2%% on 1 GPU, off)")
    ap.add_argument("--lr", type=float, default=3e-5)
    ap.add_argument("--profile-steps", type=int, default=0, help="extra steps under torch.profiler (not timed)")
    ap.add_argument("--backend", default=None, help="process-group backend override (default: nccl=RCCL on GPU)")
    ap.add_argument("--tunableop", choices=["off", "use", "tune"], default="use",
                    help="PyTorch TunableOp for the hipBLASLt GEMMs: 'use' loads the committed per-shape "
                         "solution table (tunableop/), 'tune' benchmarks new shapes during warmup and writes it")
    return ap.parse_args()


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    import dtg  # noqa: F401
    from dtg.models import build_model, resolve_config
    from dtg.parallel.data_parallel import DataParallel, FlatAdamW

    if args.tunableop != "off" and torch.cuda.is_available():
        from dtg.utils.gemm_tuning import enable_tunableop

        enable_tunableop(tune=args.tunableop == "tune")
    if args.tunableop == "tune":
        import threading

        def _heartbeat():  # tuning can run minutes inside one step: keep the job visibly alive
            t0 = time.time()
            while True:
                time.sleep(30)
                print(f"[bench] tuning GEMMs... {time.time() - t0:.0f}s", file=sys.stderr, flush=True)

        threading.Thread(target=_heartbeat, daemon=True).start()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    cuda = torch.cuda.is_available()
    # DTG_SHARED_DEVICE=1: every rank on cuda:0 (engine tests with the gloo backend on a 1-GPU box)
    dev_idx = 0 if os.environ.get("DTG_SHARED_DEVICE") == "1" else local_rank
    device = torch.device(f"cuda:{dev_idx}" if cuda else "cpu")
    if cuda:
        torch.cuda.set_device(device)
    if world > 1:
        backend = args.backend or ("nccl" if cuda else "gloo")
        dist.init_process_group(backend, device_id=device if (cuda and backend == "nccl") else None)
    torch.manual_seed(0)

    cfg = resolve_config(args.model)
    model = build_model(cfg, device=device)
    if args.parallel == "fsdp":
        from dtg.parallel.fsdp import FullyShard

        engine = FullyShard(model)
    else:
        engine = DataParallel(model, mode=args.parallel if world > 1 else "single", bucket_mb=args.bucket_mb,
                              overlap_optimizer=bool(args.overlap_optimizer))
    opt = FlatAdamW(engine, lr=args.lr)
    sched = torch.optim.lr_scheduler.CosineAnnealingLR(opt, T_max=1000, eta_min=args.lr * 1e-2)

    B, S = args.batch_size, args.seq_len
    g = torch.Generator(device=device).manual_seed(1234 + rank)
    batches = [torch.randint(0, cfg.vocab_size, (B, S), device=device, generator=g) for _ in range(4)]
    num_valid = B * (S - 1)

    def step(i):
        ids = batches[i % len(batches)]
        opt.zero_grad()
        out = model(input_ids=ids, labels=ids, num_valid=num_valid)
        engine.backward(out.loss)
        opt.step()
        sched.step()
        return out.loss

    def sync():
        if world > 1:
            dist.barrier()
        if cuda:
            torch.cuda.synchronize()

    loss = None
    for i in range(args.warmup):
        tw = time.perf_counter()
        loss = step(i)
        if cuda:
            torch.cuda.synchronize()
        print(f"[bench] warmup step {i}: {time.perf_counter() - tw:.2f}s", file=sys.stderr, flush=True)
    sync()
    if cuda:
        torch.cuda.reset_peak_memory_stats(device)
    t0 = time.perf_counter()
    for i in range(args.steps):
        loss = step(args.warmup + i)
    sync()
    elapsed = time.perf_counter() - t0
    if args.tunableop == "tune" and cuda and rank == 0:
        from dtg.utils.gemm_tuning import save_tunableop

        save_tunableop()
    el = torch.tensor([elapsed], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())
    peak_gb = torch.cuda.max_memory_allocated(device) / 2**30 if cuda else 0.0

    if args.profile_steps > 0 and cuda:
        from torch.profiler import ProfilerActivity, profile

        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
            for i in range(args.profile_steps):
                step(i)
            torch.cuda.synchronize()
        if rank == 0:
            os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
            with open(os.path.join(ROOT, "gpurun_out", "torch_profile.txt"), "w") as fp:
                fp.write(prof.key_averages().table(sort_by="cuda_time_total", row_limit=60))

    tokens = world * B * S * args.steps
    tps = tokens / elapsed
    ms = 1000 * elapsed / args.steps
    flops_tok = cfg.flops_per_token(S)
    mfu = tps * flops_tok / (world * 2.5e15) if cuda else 0.0
    if rank == 0:
        rec = {
            "metric": "tokens/sec/GPU (causal-LM pretrain) at 1/2/4/8 MI355X; FSDP peak-mem",
            "value": round(tps, 1),
            "unit": "tokens/s (whole job)",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 2),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic (uniform random token ids), random-init weights",
            "config": {"model": cfg.hf_name or args.model, "global_batch": world * B, "seq_len": S,
                       "parallelism": f"dp{world}-{engine.mode if hasattr(engine, 'mode') else args.parallel}"},
            "tokens_per_sec_per_gpu": round(tps / world, 1),
            "mfu_vs_2.5PF_dense_bf16": round(mfu, 4),
            "peak_mem_gb": round(peak_gb, 2),
            "final_loss": round(float(loss.item()), 4),
        }
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
