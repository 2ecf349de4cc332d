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

T_START = time.time()  # the run's wall clock starts here (diagnostic budget, deadline, wall_s)
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
    # ZeRO's bucket collectives: RCCL (default) or copy-engine pulls between the ranks' shared flat
    # buffers over xGMI (parallel/xgmi_dp.py); the N > 1 sweep times the other one too
    # auto (default) = the faster of the two on this job's group at one bucket, timed at startup in a
    # child job (parallel/transport.py; a first contact with cross-device IPC cannot take the measured
    # run down); recorded as dp_comm_calibration
    # RCCL by default (auto = the child-job calibration of parallel/transport.py, opt-in until a
    # multi-GPU run has validated the direct-peer paths; their evidence comes from the xGMI child
    # diagnostic after the timed region)
    ap.add_argument("--dp-comm", default="rccl", choices=["auto", "rccl", "xgmi-dma"])
    # BASELINE config 06 (Llama-3-8B TP=8 over xGMI): --tp 8 --gpus 8.  Tensor + sequence parallel
    # inside groups of --tp ranks, data parallel (--parallel) across them; a step is dp x B x S
    # tokens (the reference's TP tok/s formula, 06-tensor-parallel/train_llm.py:256).
    ap.add_argument("--tp", type=int, default=1)
    # auto = the fastest of RCCL / xGMI pull kernels / xGMI copy engines at this job's TP message size,
    # timed at startup in a child job like --dp-comm auto (opt-in, as in the trainer); the PG backend on CPU
    ap.add_argument("--tp-comm", default="rccl", choices=["auto", "rccl", "xgmi", "xgmi-dma"])
    ap.add_argument("--tp-overlap-chunks", type=int, default=2)
    ap.add_argument("--overlap-optimizer", type=int, default=0,
                    help="1: per-bucket AdamW (and ZeRO all-gather) on a side stream during backward (measured +0.2%% on 1 GPU, off)")
    ap.add_argument("--lr", type=float, default=3e-5)
    ap.add_argument("--profile-steps", type=int, default=0, help="extra steps under torch.profiler (not timed)")
    ap.add_argument("--profile-out", default="", help="torch.profiler table path (default gpurun_out/torch_profile.txt)")
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
    # N > 1 only, after the timed region: ZeRO/DDP step time rebuilt at each bucket size (MiB)
    ap.add_argument("--bucket-sweep-mb", default="64,128,256,512")
    ap.add_argument("--sweep-steps", type=int, default=3)
    ap.add_argument("--sweep-other-dp-comm", type=int, default=1,
                    help="1: the bucket sweep also times ZeRO on the other --dp-comm transport")
    # The xGMI diagnostics (the direct-peer library's collective rows and ZeRO over the copy
    # engines) run in a CHILD job launched by rank 0 after the timed region: a first contact of
    # IPC-mapped peer memory with a machine must not be able to take the measured run down.
    ap.add_argument("--xgmi-child", type=int, default=1)
    ap.add_argument("--diag-only", default="", choices=["", "xgmi", "calibrate"], help=argparse.SUPPRESS)
    # Wall-clock contract of a run (the driver kills a bench at its own limit, 600 s so far): every
    # diagnostic phase after the timed region starts only while the run is younger than
    # --diag-budget-s; at --deadline-s a watchdog prints the headline line (diagnostics done so far,
    # the rest named in diagnostic_errors) and ends every rank with exit code 0.
    ap.add_argument("--diag-budget-s", type=float, default=240.0)
    ap.add_argument("--deadline-s", type=float, default=480.0)
    ap.add_argument("--xgmi-child-timeout", type=float, default=150.0)
    ap.add_argument("--calib-child-timeout", type=float, default=120.0)
    # tests: "child-sleep:S" replaces the xGMI child job by one that sleeps S s; "hang" adds a
    # diagnostic phase that never returns
    ap.add_argument("--diag-stub", default="", help=argparse.SUPPRESS)
    # reference-mode throughput: this many extra steps under the reference's synchronising
    # LocalTimer phases (outside the timed region); 0 = off
    ap.add_argument("--ref-steps", type=int, default=3)
    # N > 1: RCCL environment preset applied before init (dtg/utils/rccl.py; exported variables win)
    ap.add_argument("--rccl-preset", default="node", choices=["node", "multinode", "none"])
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


def _batches(torch, cfg, B, S, n, device, seed):
    """n distinct batches of fresh uniform token ids, generated on the device before the timed
    region.  Uniform ids carry no learnable signal, so the loss stays near ln(vocab) for the
    whole run: a kernel whose numerics regress moves it off that value (the tripwire below),
    where four recycled batches let the model memorise them down to ~0.04 and hid any such
    regression."""
    g = torch.Generator(device=device).manual_seed(seed)
    return [torch.randint(0, cfg.vocab_size, (B, S), device=device, generator=g) for _ in range(n)]


def loss_in_band(loss: float, vocab: int) -> bool:
    """Tripwire for the synthetic run: next-token loss on uniform ids must stay within
    [ln V - 3.5, ln V + 1.5] (Llama-3-8B: 8.26 .. 13.26 around ln 128256 = 11.76)."""
    lnv = math.log(vocab)
    return math.isfinite(loss) and lnv - 3.5 < loss < lnv + 1.5


def build_job(args, torch, device, cuda, bucket_mb=None, dp_comm=None):
    """Model + engine + optimizer + scheduler of the flagship step, as the driver's command
    builds them.  `bucket_mb` overrides --bucket-mb (the N > 1 bucket-size sweep)."""
    from dtg.models import build_model, resolve_config
    from dtg.parallel.data_parallel import DataParallel, FlatAdamW

    cfg = resolve_config(args.model)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    dp_group = tp_group = xgmi = None
    dp_size, dp_rank = world, rank
    tp_comm = resolve_tp_comm(args.tp_comm, cuda)
    if args.tp > 1:
        from dtg.parallel.tensor_parallel import make_mesh

        dp_group, tp_group, dp_rank, _, dp_size = make_mesh(args.tp)
        if tp_comm != "rccl" and cuda:
            from dtg.parallel.xgmi import XgmiCommunicator
            from dtg.utils import comm as _comm

            xgmi = XgmiCommunicator(tp_group, capacity_bytes=256 << 20, device=device,
                                    gather_engine="dma" if tp_comm == "xgmi-dma" else "kernel")
            _comm.register_xgmi(tp_group, xgmi)
    model = build_model(cfg, device=device, tp_group=tp_group)
    if tp_group is not None:
        model.tp.overlap_chunks = max(1, args.tp_overlap_chunks)
    if args.parallel == "fsdp":
        from dtg.parallel.fsdp import FullyShard

        engine = FullyShard(model, group=dp_group, tp_group=tp_group, dp_comm=(dp_comm or args.dp_comm) if cuda else "rccl")
    else:
        engine = DataParallel(model, mode=args.parallel if dp_size > 1 else "single", group=dp_group, tp_group=tp_group,
                              bucket_mb=bucket_mb or args.bucket_mb, broadcast_from_rank0=tp_group is None,
                              overlap_optimizer=bool(args.overlap_optimizer),
                              dp_comm=(dp_comm or args.dp_comm) if cuda else "rccl")
    opt = FlatAdamW(engine, lr=args.lr)
    sched = torch.optim.lr_scheduler.CosineAnnealingLR(opt, T_max=1000, eta_min=args.lr * 1e-2)
    return dict(cfg=cfg, model=model, engine=engine, opt=opt, sched=sched, dp_size=dp_size, dp_rank=dp_rank,
                tp_group=tp_group, xgmi=xgmi, tp_comm=tp_comm)


def close_job(job, torch):
    eng = job["engine"]
    if hasattr(eng, "wait_param_gather"):
        eng.wait_param_gather()
    if job["xgmi"] is not None:
        torch.cuda.synchronize()
        job["xgmi"].check()
        from dtg.utils import comm as _comm

        _comm.unregister_xgmi(job["tp_group"])
        job["xgmi"].close()
    xdp = getattr(eng, "xdp", None)
    if xdp is not None:
        torch.cuda.synchronize()
        xdp.check()
    job.clear()


def resolve_tp_comm(choice: str, cuda: bool) -> str:
    """A transport still "auto" here (nothing calibrated it: CPU, one rank, a gloo rehearsal) is the
    process group's own collectives; resolve_transports() replaces "auto" by the measured pick."""
    if choice != "auto":
        return choice
    return "rccl"


def throughput_phase(args, torch, dist, device, world, rank, cuda):
    from dtg.utils.timers import make_timers

    job = build_job(args, torch, device, cuda)
    cfg, model, engine, opt, sched = job["cfg"], job["model"], job["engine"], job["opt"], job["sched"]
    dp_size, dp_rank = job["dp_size"], job["dp_rank"]

    B, S = args.batch_size, args.seq_len
    # one batch per TP group; every step (warm-up, timed, reference-timer) gets fresh ids
    n_batches = min(512, args.warmup + args.steps + args.ref_steps + max(0, args.profile_steps))
    batches = _batches(torch, cfg, B, S, n_batches, device, 1234 + dp_rank)
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
    loss_val = float(loss.item())
    if args.tunableop == "tune" and cuda and rank == 0:
        from dtg.utils.gemm_tuning import save_tunableop

        save_tunableop()
    peak_gb = torch.cuda.max_memory_allocated(device) / 2**30 if cuda else 0.0

    # Reference-mode throughput (outside the timed region): the reference's LocalTimer phases,
    # each bracketed by a device synchronize (/root/reference/01-single-gpu/train_llm.py:156-170,
    # 262-288), tok/s = 1000 * tok_per_step / sum of the phase averages.
    ref_ms = None
    if args.ref_steps > 0:
        timers = make_timers(device, sync=True)
        base = args.warmup + args.steps
        for i in range(args.ref_steps):
            with timers["data"]:
                ids = batches[(base + i) % len(batches)]
            with timers["forward"]:
                opt.zero_grad()
                out = model(input_ids=ids, labels=ids, num_valid=num_valid)
            with timers["backward"]:
                engine.backward(out.loss)
            with timers["update"]:
                opt.step()
                sched.step()
            del out
        ref_ms = {k: t.avg_elapsed_ms() for k, t in timers.items()}

    if args.profile_steps > 0 and cuda:
        from torch.profiler import ProfilerActivity, profile

        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
            for i in range(args.profile_steps):
                step(i)
            torch.cuda.synchronize()
        if rank == 0:
            out = args.profile_out or os.path.join(ROOT, "gpurun_out", "torch_profile.txt")
            os.makedirs(os.path.dirname(out), exist_ok=True)
            with open(out, "w") as fp:
                fp.write(f"# {args.profile_steps} steps; CUDA time per op and input shape\n")
                fp.write(prof.key_averages(group_by_input_shape=True).table(sort_by="cuda_time_total", row_limit=80,
                                                                           max_name_column_width=40,
                                                                           max_shapes_column_width=70))
    fake = int(os.environ.get("DTG_FAKE_WORLD", "0") or 0) > 1
    # a fake-world rehearsal computes on buffers no collective filled: its loss means nothing
    if not fake and not loss_in_band(loss_val, cfg.vocab_size):
        # NaN/inf (e.g. a wrong GEMM solution) or a loss off ln(V) on uniform ids is a numerics
        # failure, not a measurement
        raise SystemExit(f"bench.py: rank {rank} final loss {loss_val} is outside the uniform-data band around "
                         f"ln({cfg.vocab_size}) = {math.log(cfg.vocab_size):.2f}; refusing to report a throughput")
    res = dict(elapsed=elapsed, peak_gb=peak_gb, loss=loss_val, cfg=cfg, ref_ms=ref_ms,
               mode=getattr(engine, "mode", args.parallel), dp=dp_size, tp_comm=job["tp_comm"],
               dp_comm=getattr(engine, "dp_comm", "rccl"),
               replica_sum=replica_checksum(engine, torch))
    del model, engine, opt, sched, batches, loss
    close_job(job, torch)
    return res


def replica_checksum(engine, torch):
    """f64 sum of this rank's full parameter replica (DDP / ZeRO): after the step's all-gather
    every data-parallel rank must hold bit-identical weights, so the values gathered from all
    ranks must agree exactly -- a check that every collective of the timed run landed."""
    space = getattr(engine, "space", None)
    if space is None or getattr(engine, "mode", "single") not in ("ddp", "zero") or engine.tp_group is not None:
        return float("nan")
    if hasattr(engine, "wait_param_gather"):
        engine.wait_param_gather()
    buf = space.param_buf.view(-1)
    tot = torch.zeros((), dtype=torch.float64, device=buf.device)
    for i in range(0, buf.numel(), 1 << 26):  # 512 MB of f64 at a time (a whole-buffer copy is 8 B/param)
        tot += buf[i:i + (1 << 26)].double().sum()
    return float(tot.item())


def bucket_sweep(args, torch, dist, device, world, rank, cuda):
    """N > 1, after the timed region: the same step rebuilt at each gradient-bucket size of
    --bucket-sweep-mb (1 warm-up + --sweep-steps timed steps each, max over ranks), so the run
    records the curve the --bucket-mb default is chosen from.  Not part of `value`."""
    sizes = [int(x) for x in args.bucket_sweep_mb.split(",") if x.strip()]
    out = []
    B, S = args.batch_size, args.seq_len
    runs = [(mb, args.dp_comm) for mb in sizes]
    other = "xgmi-dma" if args.dp_comm == "rccl" else "rccl"
    if cuda and args.parallel == "zero" and args.sweep_other_dp_comm and (other == "rccl" or not args.xgmi_child):
        runs.append((args.bucket_mb, other))  # the other ZeRO transport at the default bucket size
    for mb, dpc in runs:
        # the sweep rebuilds the whole job per size: stop between runs once the diagnostic budget
        # is spent (every rank decides from the same broadcast clock, so all skip together)
        late = torch.tensor([float(time.time() - T_START > args.diag_budget_s)], dtype=torch.float64, device=device)
        if world > 1:
            dist.broadcast(late, src=0)
        if late.item() > 0:
            out.append({"bucket_mb": mb, "dp_comm": dpc, "skipped": "diagnostic budget spent"})
            continue
        try:
            job = build_job(args, torch, device, cuda, bucket_mb=mb, dp_comm=dpc)
        except Exception as e:  # a diagnostic row: never lose the run's JSON line over it
            out.append({"bucket_mb": mb, "dp_comm": dpc, "error": repr(e)[:300]})
            continue
        model, engine, opt = job["model"], job["engine"], job["opt"]
        ids_all = _batches(torch, job["cfg"], B, S, 1 + args.sweep_steps, device, 777 + job["dp_rank"])

        def step(ids):
            opt.zero_grad()
            out_ = model(input_ids=ids, labels=ids, num_valid=B * (S - 1))
            engine.backward(out_.loss)
            opt.step()

        step(ids_all[0])
        _sync(dist, world, cuda)
        t0 = time.perf_counter()
        for ids in ids_all[1:]:
            step(ids)
        _sync(dist, world, cuda)
        ms = torch.tensor([1000 * (time.perf_counter() - t0) / max(1, args.sweep_steps)], dtype=torch.float64,
                          device=device)
        if world > 1:
            dist.all_reduce(ms, op=dist.ReduceOp.MAX)
        # every replica must hold bit-identical weights after the steps (over the copy engines on
        # a real node: the cross-device check of the shared-buffer path, csrc/comm/xgmi.hip)
        csum = torch.tensor([replica_checksum(engine, torch)], dtype=torch.float64, device=device)
        sums = [torch.zeros_like(csum) for _ in range(world)] if world > 1 else [csum]
        if world > 1:
            dist.all_gather(sums, csum)
        sums = [float(t.item()) for t in sums]
        out.append({"bucket_mb": mb, "dp_comm": getattr(engine, "dp_comm", "rccl"),
                    "buckets": len(engine.space.buckets) if hasattr(engine, "space") else None,
                    "ms_per_step": round(float(ms.item()), 2),
                    "replicas_consistent": None if sums[0] != sums[0] else len(set(sums)) == 1})
        del model, engine, opt, ids_all, step
        close_job(job, torch)
        import gc

        gc.collect()
        if cuda:
            torch.cuda.empty_cache()
    return out


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
    profiles/r3/s22/).  Returns the child's JSON record, or None if it failed."""
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
    if cuda and 1 < world <= 8 and not args.xgmi_child:
        out.extend(_xgmi_sweep(torch, dist, device, world, cuda, [s for s in sizes if s <= 256]))
    return out


def _xgmi_sweep(torch, dist, device, world, cuda, sizes):
    """The same messages over the direct-peer xGMI library (parallel/xgmi.py), pull kernels and
    copy engines, next to RCCL's rows: the evidence --tp-comm / --dp-comm defaults rest on."""
    if not sizes:
        return []
    rows = []
    xc = None
    try:
        from dtg.parallel.xgmi import XgmiCommunicator

        from dtg.utils import comm

        xc = XgmiCommunicator(None, capacity_bytes=max(sizes) << 20, device=device)
        gen = torch.Generator(device=device).manual_seed(1000 + dist.get_rank())
        for mib in sizes:
            n = (mib << 20) // 2 // world * world
            x = torch.randn(n, device=device, generator=gen).to(torch.bfloat16)  # differs per rank
            shard = torch.empty(n // world, device=device, dtype=torch.bfloat16)
            full = torch.empty(n, device=device, dtype=torch.bfloat16)
            # cross-device correctness on a real node (every xGMI test of the suite shares one GPU):
            # the process group's result of the same message is the reference
            ref_shard = comm.reduce_scatter_dim0(x, None).float()
            ref_full = None
            for eng in ("kernel", "dma"):
                xc.gather_engine = eng
                for op, fn in (("reduce_scatter", lambda: xc.reduce_scatter_into(shard, x)),
                               ("all_gather", lambda: xc.all_gather_into(full, shard))):
                    iters = 5 if mib >= 128 else 10
                    fn()
                    _sync(dist, world, cuda)
                    if op == "reduce_scatter":  # sums in another order: bf16-rounding tolerance
                        check = {"max_rel_err": float((shard.float() - ref_shard).abs().max() /
                                                      ref_shard.abs().max().clamp_min(1e-30))}
                        ref_full = comm.all_gather_dim0(shard, None)
                    else:  # pure copies: bit-identical
                        check = {"equal": bool(torch.equal(full, ref_full))}
                    t0 = time.perf_counter()
                    for _ in range(iters):
                        fn()
                    _sync(dist, world, cuda)
                    dt = (time.perf_counter() - t0) / iters
                    rows.append({"op": f"{op}_xgmi_{eng}", "mib": mib, "us": round(dt * 1e6, 1),
                                 "busbw_gbs": round(n * 2 / dt / 1e9 * (world - 1) / world, 4), **check})
            del x, shard, full, ref_shard, ref_full
        xc.check()
    except Exception as e:  # a diagnostic: never lose the run's JSON line over it
        rows.append({"op": "xgmi", "error": repr(e)[:300]})
    finally:
        if xc is not None:
            try:
                xc.close()
            except Exception:
                pass
    return rows


_CHILD_PGIDS = set()  # process groups of running child jobs: the watchdog kills them before exiting


def _run_child(cmd, timeout, env):
    """Run a child job in its own process group; on timeout the whole group (torchrun and its
    workers) is killed.  Returns (returncode or None on timeout, stdout, stderr)."""
    import signal

    pr = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env,
                          start_new_session=True)
    _CHILD_PGIDS.add(pr.pid)
    try:
        out, err = pr.communicate(timeout=max(1.0, timeout))
        return pr.returncode, out, err
    except subprocess.TimeoutExpired:
        try:
            os.killpg(pr.pid, signal.SIGKILL)
        except ProcessLookupError:
            pass
        out, err = pr.communicate()
        return None, out, err
    finally:
        _CHILD_PGIDS.discard(pr.pid)


def _child_env():
    drop = ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK", "ROLE_WORLD_SIZE",
            "MASTER_ADDR", "MASTER_PORT", "GROUP_WORLD_SIZE", "NCCL_DEBUG", "NCCL_DEBUG_FILE", "NCCL_DEBUG_SUBSYS")
    return {k: v for k, v in os.environ.items() if k not in drop and not k.startswith("TORCHELASTIC_")}


def _child_cmd(args, world, what):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__),
           "--gpus", str(world), "--diag-only", what, "--model", args.model, "--batch-size", str(args.batch_size),
           "--seq-len", str(args.seq_len), "--bucket-mb", str(args.bucket_mb), "--coll-sweep-mb", args.coll_sweep_mb,
           "--sweep-steps", str(args.sweep_steps), "--tunableop", args.tunableop, "--parallel", args.parallel,
           "--tp", str(args.tp), "--tp-overlap-chunks", str(args.tp_overlap_chunks),
           "--dp-comm", args.dp_comm, "--tp-comm", args.tp_comm]
    if args.backend:
        cmd += ["--backend", args.backend]
    return cmd


def _child_json(rc, out, err, label, timeout):
    if rc is None:
        return {"error": f"{label} child timed out ({timeout:.0f} s)", "stderr_tail": (err or "")[-400:]}
    lines = [l for l in out.splitlines() if l.startswith("{")]
    if rc != 0 or not lines:
        return {"error": f"{label} child exited {rc}", "stderr_tail": (err or "")[-600:]}
    return json.loads(lines[-1])


def xgmi_child_diag(args, world, timeout):
    """Rank 0: `torchrun --nproc-per-node world bench.py --diag-only xgmi ...` as a child job on the
    same GPUs; returns its JSON record (or an error record).  The child times the xGMI library's
    all-gather / reduce-scatter (pull kernels and copy engines) and a ZeRO step over the copy
    engines at this run's config."""
    if args.diag_stub.startswith("child-sleep:"):
        cmd = [sys.executable, "-c", f"import time; time.sleep({float(args.diag_stub.split(':')[1])})"]
    else:
        cmd = _child_cmd(args, world, "xgmi")
    rc, out, err = _run_child(cmd, timeout, _child_env())
    return _child_json(rc, out, err, "xgmi diagnostic", timeout)


def calibrate_child(args, world, timeout):
    """Rank 0, before anything is built: `--diag-only calibrate` as a child job times RCCL against the
    xGMI transports at this job's message sizes (parallel/transport.py) and returns
    {"dp": {"choice", "table"}, "tp": {...}}.  The first contact of the xGMI library with
    cross-device IPC happens there, never in the measured processes."""
    rc, out, err = _run_child(_child_cmd(args, world, "calibrate"), timeout, _child_env())
    return _child_json(rc, out, err, "transport calibration", timeout)


def calibrate_main(args, torch, dist, device, world, rank, cuda):
    """--diag-only calibrate (the child job)."""
    from dtg.parallel import transport

    out = {}
    if args.dp_comm == "auto" and args.parallel in ("zero", "fsdp") and world // max(1, args.tp) > 1:
        group = None
        if args.tp > 1:
            from dtg.parallel.tensor_parallel import make_mesh

            group = make_mesh(args.tp)[0]
        if args.parallel == "zero":
            msg = args.bucket_mb << 20
        else:
            from dtg.models import resolve_config

            cfg = resolve_config(args.model)
            emb = cfg.vocab_size * cfg.hidden_size * (1 if cfg.tie_word_embeddings else 2)
            msg = 2 * ((cfg.num_params() - emb) // cfg.num_hidden_layers) // max(1, args.tp)
        choice, table = transport.select("dp", group, device, msg)
        out["dp"] = {"choice": choice, "table": table}
    if args.tp_comm == "auto" and args.tp > 1:
        from dtg.models import resolve_config
        from dtg.parallel.tensor_parallel import make_mesh

        cfg = resolve_config(args.model)
        tp_group = make_mesh(args.tp)[1]
        msg = transport.tp_message_bytes(args.batch_size, args.seq_len, cfg.hidden_size) // max(1, args.tp_overlap_chunks)
        choice, table = transport.select("tp", tp_group, device, msg)
        out["tp"] = {"choice": choice, "table": table}
    if rank == 0:
        print(json.dumps(out), flush=True)
    dist.barrier()
    dist.destroy_process_group()
    return 0


def resolve_transports(args, torch, dist, world, rank, cuda, backend):
    """--dp-comm / --tp-comm auto -> concrete transports on every rank.  GPU + RCCL: rank 0 runs the
    calibration child job and broadcasts its pick; otherwise (CPU, gloo rehearsals, one rank) the
    process group's own collectives.  Returns the calibration record (or None)."""
    need_dp = args.dp_comm == "auto"
    need_tp = args.tp_comm == "auto"
    if not (need_dp or need_tp):
        return None
    rec = None
    if cuda and world > 1 and backend == "nccl" and (
            (need_dp and args.parallel in ("zero", "fsdp") and world // max(1, args.tp) > 1) or (need_tp and args.tp > 1)):
        box = [None]
        if rank == 0:
            box[0] = calibrate_child(args, world, args.calib_child_timeout)
        dist.broadcast_object_list(box, src=0)
        rec = box[0]
    if need_dp:
        args.dp_comm = (rec or {}).get("dp", {}).get("choice", "rccl")
    if need_tp:
        args.tp_comm = (rec or {}).get("tp", {}).get("choice", "rccl")
    return rec


def xgmi_diag_main(args, torch, dist, device, world, rank, cuda):
    """--diag-only xgmi (the child job): xGMI collective rows + a ZeRO step on the copy engines."""
    out = {"collectives": _xgmi_sweep(torch, dist, device, world, cuda,
                                      [int(s) for s in args.coll_sweep_mb.split(",") if s.strip() and int(s) <= 256])}
    if args.parallel == "zero":
        a2 = argparse.Namespace(**vars(args))
        a2.bucket_sweep_mb, a2.sweep_other_dp_comm, a2.dp_comm = str(args.bucket_mb), 0, "xgmi-dma"
        out["zero_step"] = bucket_sweep(a2, torch, dist, device, world, rank, cuda)
    if rank == 0:
        print(json.dumps(out), flush=True)
    dist.barrier()
    dist.destroy_process_group()
    return 0


class Reporter:
    """Rank 0's one JSON line, printed exactly once: normally at the end of the run, or by the
    watchdog at --deadline-s with whatever the diagnostics have added so far."""

    def __init__(self, rank, deadline_s):
        import threading

        self.rank = rank
        self.rec = None
        self.phase = "startup"
        self.lock = threading.Lock()
        self.done = False
        self.deadline_s = deadline_s
        self.timer = threading.Thread(target=self._watch, daemon=True)
        self.timer.start()

    def _watch(self):
        time.sleep(max(0.0, T_START + self.deadline_s - time.time()))
        import signal

        for pg in list(_CHILD_PGIDS):
            try:
                os.killpg(pg, signal.SIGKILL)
            except (ProcessLookupError, PermissionError):
                pass
        with self.lock:
            if self.done:
                return
            if self.rec is None:  # the timed region never finished: nothing to report
                print(f"[bench] rank {self.rank}: deadline {self.deadline_s:.0f} s reached in phase "
                      f"'{self.phase}' before the timed region finished", file=sys.stderr, flush=True)
                os._exit(3)
            self.rec.setdefault("diagnostic_errors", {})[self.phase] = (
                f"still running at the {self.deadline_s:.0f} s deadline: the line was printed by the watchdog")
            self._print_locked()
        os._exit(0)

    def _print_locked(self):
        self.done = True
        if self.rank == 0:
            self.rec["wall_s"] = round(time.time() - T_START, 1)
            print(json.dumps(self.rec), flush=True)

    def emit(self):
        with self.lock:
            if not self.done:
                self._print_locked()


def _load_rccl_module():
    import importlib.util

    path = os.path.join(ROOT, "lambda-labs_distributed-training-guide_amd", "utils", "rccl.py")
    spec = importlib.util.spec_from_file_location("_dtg_rccl_preinit", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    # DTG_FAKE_WORLD=N: rehearsal of rank 0 of an N-rank job on one GPU; the other ranks are
    # PyTorch's fake process group (collectives return at once).  Shapes, shard layouts, kernels
    # and memory are those of the real N-rank job; the time excludes communication and is labelled.
    fake_world = int(os.environ.get("DTG_FAKE_WORLD", "0") or 0)
    if fake_world > 1 and ("TORCHELASTIC_RUN_ID" in os.environ or int(os.environ.get("WORLD_SIZE", "1") or 1) > 1):
        raise SystemExit("bench.py: DTG_FAKE_WORLD is set inside a multi-rank launch; unset it "
                         "(a rehearsal is one process)")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ and fake_world <= 1:
        return self_launch(args, argv)

    # A real multi-rank job (RCCL): the node preset (utils/rccl.py; never overrides an exported
    # variable) goes in before anything initialises HIP, and RCCL's INIT/GRAPH log is captured
    # to a per-rank file so the JSON line can say what RCCL built (transport, channels).
    multi = int(os.environ.get("WORLD_SIZE", "1")) > 1 and fake_world <= 1
    rccl_log = rccl_applied = None
    if multi and args.rccl_preset != "none":
        _rccl = _load_rccl_module()  # stdlib-only: importing it does not touch the GPU
        rccl_applied = _rccl.apply_preset(args.rccl_preset)
        rccl_log = _rccl.arm_log(f"rank{os.environ.get('RANK', '0')}_{os.getpid()}")

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
    if args.diag_only == "xgmi":
        return xgmi_diag_main(args, torch, dist, device, world, rank, cuda)
    if args.diag_only == "calibrate":
        return calibrate_main(args, torch, dist, device, world, rank, cuda)

    reporter = Reporter(rank, args.deadline_s)
    phase_s = {}
    t_ph = time.time()
    reporter.phase = "transport_calibration"
    calib = resolve_transports(args, torch, dist, world, rank, cuda, backend)
    phase_s["startup_and_calibration"] = round(time.time() - T_START, 1)
    reporter.phase = "throughput"
    t_ph = time.time()
    res = throughput_phase(args, torch, dist, device, world, rank, cuda)
    phase_s["throughput"] = round(time.time() - t_ph, 1)
    gc.collect()
    if cuda:
        torch.cuda.empty_cache()

    # ---- the headline, gathered and built BEFORE any diagnostic: from here on the line is printed
    # whatever a diagnostic does (error -> diagnostic_errors; hang -> the watchdog at --deadline-s)
    def gather(vals):
        mine = torch.tensor(vals, dtype=torch.float64, device=device)
        if world > 1 and fake_world <= 1:
            allv = [torch.zeros_like(mine) for _ in range(world)]
            dist.all_gather(allv, mine)
            return [v.cpu().tolist() for v in allv]
        return [mine.cpu().tolist()]  # one rank, or the other ranks do not exist (fake world)

    ref_keys = ("data", "forward", "backward", "update")
    rows = gather([res["elapsed"], float(dev_idx), float(res["peak_gb"]), sum(res["ref_ms"].values()) if res["ref_ms"]
                   else 0.0, res["replica_sum"]] + ([res["ref_ms"][k] for k in ref_keys] if res["ref_ms"] else [0.0] * 4))
    bus = None
    if cuda:
        bus = getattr(torch.cuda.get_device_properties(device), "pci_bus_id", None)
    elapsed = max(r[0] for r in rows)  # the slowest rank bounds the job
    cfg = res["cfg"]
    B, S = args.batch_size, args.seq_len
    dp = res["dp"]
    tps = dp * B * S * args.steps / elapsed
    ms = 1000 * elapsed / args.steps
    mfu = tps * cfg.flops_per_token(S) / (world * 2.5e15) if cuda else 0.0
    # TP collectives: "rccl" means the process group's own backend (gloo in CPU / shared-GPU rehearsals)
    tp_comm = res["tp_comm"]
    tp_comm_label = tp_comm if tp_comm != "rccl" else ("rccl" if backend in (None, "nccl") else backend)
    rec = {}
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
                       "parallelism": f"dp{dp}-{res['mode']}" + ("-xgmi-dma" if res["dp_comm"] == "xgmi-dma" else "")
                                      + (f"-tp{args.tp}-{tp_comm_label}" if args.tp > 1 else "")},
            "tokens_per_sec_per_gpu": round(tps / world, 1),
            "mfu_vs_2.5PF_dense_bf16": round(mfu, 4),
            "peak_mem_gb": round(max(r[2] for r in rows), 2),
            "final_loss": round(res["loss"], 4) if math.isfinite(res["loss"]) else None,
            "world_size_seen_by_pg": pg_world,
            "backend": backend or "none",
            "rank_devices": [int(r[1]) for r in rows],
            "rank0_pci_bus_id": bus,
            "rank_ms_per_step": {"max": round(ms, 2), "min": round(1000 * min(r[0] for r in rows) / args.steps, 2)},
            "loss_band": [round(math.log(cfg.vocab_size) - 3.5, 2), round(math.log(cfg.vocab_size) + 1.5, 2)],
            "phase_s": phase_s,
        }
        if res["ref_ms"]:
            # the reference's own tok/s (synchronised LocalTimer phases, slowest rank)
            rec["tok_s_reference_timers"] = round(1000 * dp * B * S / max(r[3] for r in rows), 1)
            rec["reference_timer_ms"] = {k: round(max(r[5 + j] for r in rows), 2) for j, k in enumerate(ref_keys)}
            rec["reference_timer_steps"] = args.ref_steps
        sums = [r[4] for r in rows]
        if world > 1 and fake_world <= 1 and all(math.isfinite(x) for x in sums):
            # every data-parallel replica must hold bit-identical weights after the last step
            rec["replicas_consistent"] = len(set(sums)) == 1
        if fake_world > 1:
            rec["metric"] = "REHEARSAL (not a measurement of the job): " + METRIC
            rec["rehearsal"] = (f"rank 0 of a {world}-rank job alone on one GPU, other ranks a fake process "
                                "group: communication not included, value = one rank's compute rate x world")
        if calib is not None:
            for k in ("dp", "tp"):
                if k in calib:
                    rec[f"{k}_comm_calibration"] = calib[k]
            if "error" in calib:
                rec["transport_calibration_error"] = calib
        if multi and backend == "nccl":
            rec["rccl"] = _load_rccl_module().diagnose(rccl_log)
            rec["rccl"]["preset_applied"] = rccl_applied
    reporter.rec = rec
    diag_errors = {}

    def in_budget(collective=True):
        """Start the next diagnostic only while the run is younger than --diag-budget-s (all ranks
        decide together on the oldest rank's clock)."""
        age = time.time() - T_START
        if collective and world > 1 and fake_world <= 1:
            t = torch.tensor([age], dtype=torch.float64, device=device)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            age = float(t.item())
        return age < args.diag_budget_s

    def phase(name, fn, collective=True):
        if not in_budget(collective):
            diag_errors[name] = f"skipped: run older than the {args.diag_budget_s:.0f} s diagnostic budget"
            if rank == 0:
                rec.setdefault("diagnostic_errors", {})[name] = diag_errors[name]
            return None
        reporter.phase = name
        t0 = time.time()
        try:
            return fn()
        except Exception as e:  # noqa: BLE001 - recorded in the line, never loses the measurement
            diag_errors[name] = repr(e)[:300]
            if rank == 0:
                rec.setdefault("diagnostic_errors", {})[name] = diag_errors[name]
            gc.collect()
            if cuda:
                torch.cuda.empty_cache()
            return None
        finally:
            phase_s[name] = round(time.time() - t0, 1)

    # ---- after the timed region: diagnostics of the multi-rank run (none of this is in `value`),
    # cheapest and safest first; the xGMI child job (a first contact with cross-device IPC) last
    if multi and args.coll_sweep_mb:
        coll = phase("collectives", lambda: collective_sweep(args, torch, dist, device, world, cuda))
        if coll is not None and rank == 0:
            rec["collectives"] = coll
    if multi and args.bucket_sweep_mb and args.parallel in ("ddp", "zero") and args.tp == 1:
        sweep = phase("bucket_sweep", lambda: bucket_sweep(args, torch, dist, device, world, rank, cuda))
        if sweep is not None and rank == 0:
            rec["bucket_sweep"] = sweep
    if args.diag_stub == "hang":
        phase("stub_hang", lambda: time.sleep(10 ** 6))
    if args.fsdp_mem_steps > 0:
        mem = phase("fsdp_mem", lambda: fsdp_memory_phase(args, torch, dist, device, world, rank, cuda))
        gc.collect()
        mrows = gather([mem["valley"], mem["peak"], mem["ms"]] if mem else [-1.0, -1.0, -1.0])
        if rank == 0 and all(r[0] >= 0 for r in mrows):
            rec["fsdp_mem"] = {"model": mem["model"], "batch_per_gpu": args.fsdp_mem_batch,
                               "seq_len": args.fsdp_mem_seq, "wrap": f"size>={args.numel_to_wrap}",
                               "valley_gb_max_rank": round(max(r[0] for r in mrows), 2),
                               "peak_gb_max_rank": round(max(r[1] for r in mrows), 2),
                               "ms_per_step": round(max(r[2] for r in mrows), 1),
                               "reference_a100x8": {"valley_gb": 8, "peak_gb": 74}}
            rec["fsdp_peak_mem_gb"] = rec["fsdp_mem"]["peak_gb_max_rank"]
    if args.fsdp_mem_steps > 0 and cuda and rank == 0 and world < args.fsdp_mem_world:
        torch.cuda.empty_cache()
        mem_one = phase("fsdp_mem_one_rank", lambda: fsdp_mem_one_rank(args), collective=False)
        if mem_one is not None:
            rec["fsdp_mem_one_rank_of_w"] = {"world": mem_one["world"], "valley_gb": mem_one["valley_gib"],
                                             "peak_gb": mem_one["peak_gib"], "method": "rank 0 alone, other ranks a "
                                             "fake process group (tools/fsdp_mem_one_rank.py)",
                                             "reference_a100x8": {"valley_gb": 8, "peak_gb": 74}}
    run_child = multi and args.xgmi_child and world <= 8 and (cuda or args.diag_stub.startswith("child-sleep:"))
    if run_child:
        gc.collect()
        if cuda:
            torch.cuda.empty_cache()
        remaining = T_START + args.deadline_s - 30 - time.time()
        timeout = min(args.xgmi_child_timeout, remaining)
        box = [None]
        if rank == 0:
            box[0] = phase("xgmi_child", lambda: xgmi_child_diag(args, world, timeout), collective=False) \
                if timeout > 10 else None
            if timeout <= 10:
                rec.setdefault("diagnostic_errors", {})["xgmi_child"] = "skipped: too close to the deadline"
        dist.barrier()
        if rank == 0 and box[0] is not None:
            rec["xgmi_diag"] = box[0]
            if "error" in box[0]:
                rec.setdefault("diagnostic_errors", {})["xgmi_child"] = box[0]["error"]
    reporter.phase = "report"
    reporter.emit()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
