#!/usr/bin/env python3
"""Headline benchmark: causal-LM pretraining throughput on MI355X (BASELINE.json metric).

    python bench.py --gpus N --steps K --warmup W
        N=1: runs in this process.
        N>1 without a launcher: starts `torch.distributed.run --nproc-per-node N` as a CHILD
        process (nothing in this parent touches the GPU) and exits with its code, so the same
        command measures N ranks, one per GPU, over RCCL.
    torchrun --nproc-per-node N bench.py --gpus N ...
        one rank per GPU; the process group must see exactly N ranks (asserted).

Config: Llama-3-8B (bundled config, random init, pure bf16 params/grads/AdamW states as in the
reference), synthetic token data, seq 1024, fixed per-GPU micro-batch (weak scaling).  Every
timed step does the full work: forward, backward with overlapped bucketed gradient
reduce-scatter, fused AdamW on the local shard, parameter all-gather and the cosine LR step.
K steps are bracketed by barrier + device synchronize on both sides; the slowest rank's time is
reported.  Rank 0 prints one JSON line (value = whole-job tokens/s).

"FSDP peak-mem" half of the metric: after the timed throughput phase the ZeRO model is freed
and a short FSDP (FULL_SHARD, size-based wrap at --numel-to-wrap) phase runs the reference's
memory-table config (Llama-2-7B, batch 10, seq 1024: /root/reference/04-fully-sharded-data-parallel/
README.md:271-281) over the same ranks; its per-rank valley (allocated at the end of an
iteration) and peak (max allocated during it) are reported, max over ranks.  That phase is
outside the timed region and does not affect `value`.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "tokens/sec/GPU (causal-LM pretrain) at 1/2/4/8 MI355X; FSDP peak-mem"


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--batch-size", type=int, default=16, help="per-GPU micro-batch (sequences)")
    ap.add_argument("--seq-len", type=int, default=1024)
    ap.add_argument("--parallel", default="zero", choices=["ddp", "zero", "fsdp"])
    ap.add_argument("--bucket-mb", type=int, default=256)
    # BASELINE config 06 (Llama-3-8B TP=8 over xGMI): --tp 8 --gpus 8.  Tensor + sequence parallel
    # inside groups of --tp ranks, data parallel (--parallel) across them; a step is dp x B x S
    # tokens (the reference's TP tok/s formula, 06-tensor-parallel/train_llm.py:256).
    ap.add_argument("--tp", type=int, default=1)
    ap.add_argument("--tp-comm", default="rccl", choices=["rccl", "xgmi", "xgmi-dma"])
    ap.add_argument("--tp-overlap-chunks", type=int, default=2)
    ap.add_argument("--overlap-optimizer", type=int, default=0,
                    help="1: per-bucket AdamW (and ZeRO all-gather) on a side stream during backward (measured +0.2%% on 1 GPU, off)")
    ap.add_argument("--lr", type=float, default=3e-5)
    ap.add_argument("--profile-steps", type=int, default=0, help="extra steps under torch.profiler (not timed)")
    ap.add_argument("--backend", default=None, help="process-group backend override (default: nccl=RCCL on GPU)")
    ap.add_argument("--tunableop", choices=["off", "use", "tune"], default="use",
                    help="PyTorch TunableOp for the hipBLASLt GEMMs: 'use' loads the committed per-shape "
                         "solution table (tunableop/), 'tune' benchmarks new shapes during warmup and writes it")
    # FSDP memory phase (not timed into `value`)
    ap.add_argument("--fsdp-mem-model", default="llama-2-7b")
    ap.add_argument("--fsdp-mem-batch", type=int, default=10)
    ap.add_argument("--fsdp-mem-seq", type=int, default=1024)
    ap.add_argument("--fsdp-mem-steps", type=int, default=3, help="0 skips the FSDP memory phase")
    ap.add_argument("--fsdp-mem-world", type=int, default=8,
                    help="run with fewer ranks than this: also measure one rank of a job of this size "
                         "(tools/fsdp_mem_one_rank.py: the other ranks are a fake process group), the "
                         "reference's 8-GPU memory row; 0 = off")
    ap.add_argument("--numel-to-wrap", type=int, default=100_000_000)
    # After the timed region, N > 1 only: RCCL reduce-scatter / all-gather / all-reduce bus
    # bandwidth at these message sizes (MiB), so the multi-GPU run also measures the curve the
    # 256 MiB gradient-bucket default is chosen from.  Empty string = off.
    ap.add_argument("--coll-sweep-mb", default="16,64,256,1024")
    return ap.parse_args(argv)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def self_launch(args, argv) -> int:
    """N ranks without an external launcher: torchrun as a child process (never exec from a
    process that may have touched the GPU), one rank per GPU, rendezvous on 127.0.0.1."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "1")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def _sync(dist, world, cuda):
    if world > 1:
        dist.barrier()
    if cuda:
        import torch

        torch.cuda.synchronize()


def throughput_phase(args, torch, dist, device, world, rank, cuda):
    from dtg.models import build_model, resolve_config
    from dtg.parallel.data_parallel import DataParallel, FlatAdamW

    cfg = resolve_config(args.model)
    dp_group = tp_group = xgmi = None
    dp_size, dp_rank = world, rank
    if args.tp > 1:
        from dtg.parallel.tensor_parallel import make_mesh

        dp_group, tp_group, dp_rank, _, dp_size = make_mesh(args.tp)
        if args.tp_comm != "rccl" and cuda:
            from dtg.parallel.xgmi import XgmiCommunicator
            from dtg.utils import comm as _comm

            xgmi = XgmiCommunicator(tp_group, capacity_bytes=256 << 20, device=device,
                                    gather_engine="dma" if args.tp_comm == "xgmi-dma" else "kernel")
            _comm.register_xgmi(tp_group, xgmi)
    model = build_model(cfg, device=device, tp_group=tp_group)
    if tp_group is not None:
        model.tp.overlap_chunks = max(1, args.tp_overlap_chunks)
    if args.parallel == "fsdp":
        from dtg.parallel.fsdp import FullyShard

        engine = FullyShard(model, group=dp_group, tp_group=tp_group)
    else:
        engine = DataParallel(model, mode=args.parallel if dp_size > 1 else "single", group=dp_group, tp_group=tp_group,
                              bucket_mb=args.bucket_mb, broadcast_from_rank0=tp_group is None,
                              overlap_optimizer=bool(args.overlap_optimizer))
    opt = FlatAdamW(engine, lr=args.lr)
    sched = torch.optim.lr_scheduler.CosineAnnealingLR(opt, T_max=1000, eta_min=args.lr * 1e-2)

    B, S = args.batch_size, args.seq_len
    g = torch.Generator(device=device).manual_seed(1234 + dp_rank)  # one batch per TP group
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

    loss = None
    for i in range(args.warmup):
        tw = time.perf_counter()
        loss = step(i)
        if cuda:
            torch.cuda.synchronize()
        print(f"[bench] rank {rank} warmup step {i}: {time.perf_counter() - tw:.2f}s", file=sys.stderr, flush=True)
    _sync(dist, world, cuda)
    if cuda:
        torch.cuda.reset_peak_memory_stats(device)
    t0 = time.perf_counter()
    for i in range(args.steps):
        loss = step(args.warmup + i)
    _sync(dist, world, cuda)
    elapsed = time.perf_counter() - t0
    if args.tunableop == "tune" and cuda and rank == 0:
        from dtg.utils.gemm_tuning import save_tunableop

        save_tunableop()
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
    res = dict(elapsed=elapsed, peak_gb=peak_gb, loss=float(loss.item()), cfg=cfg,
               mode=getattr(engine, "mode", args.parallel), dp=dp_size)
    if not math.isfinite(res["loss"]) and int(os.environ.get("DTG_FAKE_WORLD", "0") or 0) <= 1:
        # a step that produced NaN/inf (e.g. a wrong GEMM solution) is not a measurement
        # (a fake-world rehearsal computes on buffers no collective filled: its loss means nothing)
        raise SystemExit(f"bench.py: rank {rank} final loss is {res['loss']}; refusing to report a throughput")
    if hasattr(engine, "wait_param_gather"):
        engine.wait_param_gather()
    if xgmi is not None:
        torch.cuda.synchronize()
        xgmi.check()
        from dtg.utils import comm as _comm

        _comm.unregister_xgmi(tp_group)
        xgmi.close()
    del model, engine, opt, sched, batches, loss
    return res


def fsdp_memory_phase(args, torch, dist, device, world, rank, cuda):
    """Valley / peak allocated GB per rank of FSDP FULL_SHARD on the reference's memory-table
    config (chapter 04).  Meta-device init: units are materialised one at a time."""
    from dtg.models import build_model, resolve_config
    from dtg.parallel.data_parallel import FlatAdamW
    from dtg.parallel.fsdp import FullyShard

    cfg = resolve_config(args.fsdp_mem_model)
    with torch.device("meta"):
        model = build_model(cfg, init=False)
    engine = FullyShard(model, policy="size", min_num_params=args.numel_to_wrap, device=device)
    opt = FlatAdamW(engine, lr=args.lr)
    B, S = args.fsdp_mem_batch, args.fsdp_mem_seq
    g = torch.Generator(device=device).manual_seed(99 + rank)
    ids = torch.randint(0, cfg.vocab_size, (B, S), device=device, generator=g)
    gb = 2**30
    valley = peak = 0.0
    _sync(dist, world, cuda)
    t0 = time.perf_counter()
    for i in range(args.fsdp_mem_steps):
        if cuda:
            torch.cuda.synchronize()
            torch.cuda.reset_peak_memory_stats(device)
        out = model(input_ids=ids, labels=ids, num_valid=B * (S - 1))
        engine.backward(out.loss)
        opt.step()
        opt.zero_grad()
        del out
        if cuda:
            torch.cuda.synchronize()
            peak = torch.cuda.max_memory_allocated(device) / gb
            valley = torch.cuda.memory_allocated(device) / gb
    _sync(dist, world, cuda)
    ms = 1000 * (time.perf_counter() - t0) / max(1, args.fsdp_mem_steps)
    del model, engine, opt, ids
    return dict(valley=valley, peak=peak, ms=ms, model=cfg.hf_name or args.fsdp_mem_model)


def fsdp_mem_one_rank(args):
    """Valley / peak of ONE rank of an --fsdp-mem-world-rank FSDP job on this GPU: a child process
    (tools/fsdp_mem_one_rank.py) runs rank 0 with a fake process group for the other ranks --
    exact allocations, meaningless numerics (validated against real W = 1/2/4 runs,
    profiles/r3_s22/).  Returns the child's JSON record, or None if it failed."""
    cmd = [sys.executable, os.path.join(ROOT, "tools", "fsdp_mem_one_rank.py"), "--world", str(args.fsdp_mem_world),
           "--model", args.fsdp_mem_model, "--batch", str(args.fsdp_mem_batch), "--seq", str(args.fsdp_mem_seq),
           "--numel-to-wrap", str(args.numel_to_wrap), "--steps", str(max(2, args.fsdp_mem_steps))]
    try:
        # the child is a one-process job of its own: none of this run's rank / fake-world env
        env = {k: v for k, v in os.environ.items()
               if k not in ("DTG_FAKE_WORLD", "WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE",
                            "GROUP_RANK", "ROLE_RANK", "MASTER_ADDR", "MASTER_PORT", "TORCHELASTIC_RUN_ID")}
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env)
        lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
        if r.returncode == 0 and lines:
            return json.loads(lines[-1])
        print(f"[bench] fsdp one-rank memory run failed ({r.returncode}): {r.stderr[-500:]}", file=sys.stderr)
    except subprocess.TimeoutExpired:
        print("[bench] fsdp one-rank memory run timed out", file=sys.stderr)
    return None


def collective_sweep(args, torch, dist, device, world, cuda):
    """[{op, mib, us, busbw_gbs}] measured on every rank (rank 0's numbers reported), nccl-tests
    bus-bandwidth conventions: reduce-scatter / all-gather x (W-1)/W, all-reduce x 2(W-1)/W."""
    sizes = [int(x) for x in args.coll_sweep_mb.split(",") if x.strip()]
    out = []
    dt_ = torch.bfloat16 if cuda else torch.float32
    esz = 2 if cuda else 4
    for mib in sizes:
        n = (mib << 20) // esz // world * world
        x = torch.randn(n, device=device).to(dt_)
        shard = torch.empty(n // world, device=device, dtype=dt_)
        full = torch.empty(n, device=device, dtype=dt_)
        ops = {"reduce_scatter": (lambda: dist.reduce_scatter_tensor(shard, x), (world - 1) / world),
               "all_gather": (lambda: dist.all_gather_into_tensor(full, shard), (world - 1) / world),
               "all_reduce": (lambda: dist.all_reduce(x), 2 * (world - 1) / world)}
        if dist.get_backend() == "gloo":  # gloo (CPU / shared-GPU rehearsals) has no reduce-scatter
            ops.pop("reduce_scatter")
        for op, (fn, factor) in ops.items():
            iters = 5 if mib >= 256 else 10
            fn()
            _sync(dist, world, cuda)
            t0 = time.perf_counter()
            for _ in range(iters):
                fn()
            _sync(dist, world, cuda)
            dt = (time.perf_counter() - t0) / iters
            out.append({"op": op, "mib": mib, "us": round(dt * 1e6, 1),
                        "busbw_gbs": round((n * esz) / dt / 1e9 * factor, 4)})
        del x, shard, full
    return out


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    # DTG_FAKE_WORLD=N: rehearsal of rank 0 of an N-rank job on one GPU; the other ranks are
    # PyTorch's fake process group (collectives return at once).  Shapes, shard layouts, kernels
    # and memory are those of the real N-rank job; the time excludes communication and is labelled.
    fake_world = int(os.environ.get("DTG_FAKE_WORLD", "0") or 0)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ and fake_world <= 1:
        return self_launch(args, argv)

    import gc

    import torch
    import torch.distributed as dist

    import dtg  # noqa: F401

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
    if fake_world > 1:
        os.environ.update(WORLD_SIZE=str(fake_world), RANK="0", LOCAL_RANK="0",
                          LOCAL_WORLD_SIZE=str(min(fake_world, 8)))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
    cuda = torch.cuda.is_available()
    # DTG_SHARED_DEVICE=1: every rank on cuda:0 (engine tests with the gloo backend on a 1-GPU box)
    dev_idx = 0 if os.environ.get("DTG_SHARED_DEVICE") == "1" else local_rank
    if cuda and os.environ.get("DTG_SHARED_DEVICE") != "1":
        assert local_rank < torch.cuda.device_count(), \
            f"local rank {local_rank} has no GPU (device_count={torch.cuda.device_count()})"
    device = torch.device(f"cuda:{dev_idx}" if cuda else "cpu")
    if cuda:
        torch.cuda.set_device(device)
    backend = None
    if world > 1 and fake_world > 1:
        from torch.testing._internal.distributed.fake_pg import FakeStore

        backend = "fake"
        dist.init_process_group("fake", store=FakeStore(), rank=0, world_size=world)
    elif world > 1:
        backend = args.backend or ("nccl" if cuda else "gloo")
        dist.init_process_group(backend, device_id=device if (cuda and backend == "nccl") else None)
        assert dist.get_world_size() == args.gpus, (dist.get_world_size(), args.gpus)
    pg_world = dist.get_world_size() if dist.is_initialized() else 1
    torch.manual_seed(0)

    res = throughput_phase(args, torch, dist, device, world, rank, cuda)
    gc.collect()
    if cuda:
        torch.cuda.empty_cache()
    coll = collective_sweep(args, torch, dist, device, world, cuda) if (world > 1 and fake_world <= 1 and args.coll_sweep_mb) else None
    mem = None
    if args.fsdp_mem_steps > 0:
        mem = fsdp_memory_phase(args, torch, dist, device, world, rank, cuda)
        gc.collect()
    mem_one = None
    if args.fsdp_mem_steps > 0 and cuda and rank == 0 and world < args.fsdp_mem_world:
        torch.cuda.empty_cache()
        mem_one = fsdp_mem_one_rank(args)

    # per-rank facts, gathered to rank 0: elapsed, device ordinal, PCI bus, peaks
    me = [res["elapsed"], float(dev_idx), float(res["peak_gb"]),
          mem["valley"] if mem else 0.0, mem["peak"] if mem else 0.0, mem["ms"] if mem else 0.0]
    mine = torch.tensor(me, dtype=torch.float64, device=device)
    if world > 1 and fake_world > 1:
        rows = [mine.cpu().tolist()]  # the other ranks do not exist
    elif world > 1:
        allv = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(allv, mine)
        rows = [v.cpu().tolist() for v in allv]
    else:
        rows = [mine.cpu().tolist()]
    bus = None
    if cuda:
        p = torch.cuda.get_device_properties(device)
        bus = getattr(p, "pci_bus_id", None)
    elapsed = max(r[0] for r in rows)  # the slowest rank bounds the job

    cfg = res["cfg"]
    B, S = args.batch_size, args.seq_len
    dp = res["dp"]
    tokens = dp * B * S * args.steps
    tps = tokens / elapsed
    ms = 1000 * elapsed / args.steps
    flops_tok = cfg.flops_per_token(S)
    mfu = tps * flops_tok / (world * 2.5e15) if cuda else 0.0
    # TP collectives: "rccl" means the process group's own backend (gloo in CPU / shared-GPU rehearsals)
    tp_comm_label = args.tp_comm if args.tp_comm != "rccl" else ("rccl" if backend in (None, "nccl") else backend)
    if rank == 0:
        rec = {
            "metric": METRIC,
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
            "config": {"model": cfg.hf_name or args.model, "global_batch": dp * B, "seq_len": S,
                       "parallelism": f"dp{dp}-{res['mode']}" + (f"-tp{args.tp}-{tp_comm_label}" if args.tp > 1 else "")},
            "tokens_per_sec_per_gpu": round(tps / world, 1),
            "mfu_vs_2.5PF_dense_bf16": round(mfu, 4),
            "peak_mem_gb": round(max(r[2] for r in rows), 2),
            "final_loss": round(res["loss"], 4) if math.isfinite(res["loss"]) else None,
            "world_size_seen_by_pg": pg_world,
            "backend": backend or "none",
            "rank_devices": [int(r[1]) for r in rows],
            "rank0_pci_bus_id": bus,
            "rank_ms_per_step": {"max": round(1000 * elapsed / args.steps, 2),
                                 "min": round(1000 * min(r[0] for r in rows) / args.steps, 2)},
        }
        if fake_world > 1:
            rec["metric"] = "REHEARSAL (not a measurement of the job): " + METRIC
            rec["rehearsal"] = (f"rank 0 of a {world}-rank job alone on one GPU, other ranks a fake process "
                                "group: communication not included, value = one rank's compute rate x world")
        if coll is not None and fake_world <= 1:
            rec["collectives"] = coll
        if mem is not None:
            rec["fsdp_mem"] = {"model": mem["model"], "batch_per_gpu": args.fsdp_mem_batch,
                               "seq_len": args.fsdp_mem_seq, "wrap": f"size>={args.numel_to_wrap}",
                               "valley_gb_max_rank": round(max(r[3] for r in rows), 2),
                               "peak_gb_max_rank": round(max(r[4] for r in rows), 2),
                               "ms_per_step": round(max(r[5] for r in rows), 1),
                               "reference_a100x8": {"valley_gb": 8, "peak_gb": 74}}
            rec["fsdp_peak_mem_gb"] = rec["fsdp_mem"]["peak_gb_max_rank"]
        if mem_one is not None:
            rec["fsdp_mem_one_rank_of_w"] = {"world": mem_one["world"], "valley_gb": mem_one["valley_gib"],
                                             "peak_gb": mem_one["peak_gib"], "method": "rank 0 alone, other ranks a "
                                             "fake process group (tools/fsdp_mem_one_rank.py)",
                                             "reference_a100x8": {"valley_gb": 8, "peak_gb": 74}}
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
