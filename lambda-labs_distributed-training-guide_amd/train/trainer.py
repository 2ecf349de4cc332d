"""The chaptered training driver: one implementation, eight entry points.

Every chapter's `train_llm.py` calls `run("<chapter>")`.  The loop keeps the reference's
behaviour -- epochs over a (distributed) DataLoader, phase timers data/forward/backward/update,
skip-ahead resume that still consumes batches, the metric record every `--log-freq` steps and a
checkpoint every `--ckpt-freq` steps -- on top of this framework's engines:

  rime  single GPU, Llama-3.2-3B + 28,683 tokens, packed 8192-token rows, varlen attention
  01    single device (GPU, or CPU for the GPT-2 plumbing run)
  02    data parallel: ZeRO (default, the reference's sharded optimizer) or DDP, bucketed RCCL
  04    FSDP, size-based wrap (--numel-to-wrap), optional CPU offload, meta-device init
  05    FSDP, transformer wrap + activation checkpointing + CPU offload (405B recipe)
  06    tensor + sequence parallel over the node's GPUs, data parallel across nodes
  07    2-D: FSDP over dp x tensor parallel over tp (--tp)
  deepspeed  the alternative-framework chapter: ds_config.json keys mapped onto these engines
"""
from __future__ import annotations

import json
import logging
import math
import os
import random
import time
from pathlib import Path

import torch
from tqdm import tqdm

from .. import data as dtg_data
from ..models import build_model, count_valid_labels, resolve_config
from ..parallel.checkpointing import apply_activation_checkpointing, checkpointed_count
from ..parallel.data_parallel import DataParallel, FlatAdamW
from ..utils import comm as ucomm
from ..utils import dist as udist
from ..utils.metrics import MI355X_BF16_DENSE_FLOPS, MetricSink, get_mem_stats, wandb_init_kwargs
from ..utils.timers import make_timers
from .checkpoint import CheckpointManager, has_checkpoint, new_state, recover_checkpoint
from .cli import get_parser

LOGGER = logging.getLogger("dtg")


def _deepspeed_overrides(args):
    """Map the ds_config.json keys used by the reference onto this framework."""
    cfg = {}
    if args.deepspeed_config:
        with open(args.deepspeed_config) as fp:
            cfg = json.load(fp)
    args.batch_size = int(cfg.get("train_micro_batch_size_per_gpu", 1))
    opt = cfg.get("optimizer", {}).get("params", {})
    if "lr" in opt:
        args.lr = float(opt["lr"])
    args.betas = tuple(opt.get("betas", (0.9, 0.999)))
    args.eps = float(opt.get("eps", 1e-8))
    args.weight_decay = float(opt.get("weight_decay", 0.01))
    sch = cfg.get("scheduler", {})
    args.ds_scheduler = sch
    zero = cfg.get("zero_optimization", {})
    args.zero_stage = int(zero.get("stage", 3))
    off = (zero.get("offload_optimizer") or {}).get("device", "none")
    args.cpu_offload = "on" if (off == "cpu" and args.zero_stage == 3) else "off"
    # ZeRO-Offload (optimizer only) keeps parameters on the device; offload_param moves them too
    args.offload_params = "on" if (zero.get("offload_param") or {}).get("device", "none") == "cpu" else "off"
    args.grad_accum = int(cfg.get("gradient_accumulation_steps", args.grad_accum))
    return args


def _offload_params(args, model, dp_group, device) -> bool:
    """--offload-params on|off|auto for CPU offload.  auto (default): keep the bf16 parameter
    shard resident in HBM when it takes at most a third of the device's memory -- on a 288 GB
    MI355X that is every model up to ~430 B parameters per 8 GPUs -- and offload it too beyond."""
    mode = getattr(args, "offload_params", "auto")
    if mode != "auto":
        return mode == "on"
    n = sum(p.numel() for p in model.parameters())
    w = torch.distributed.get_world_size(dp_group) if torch.distributed.is_initialized() else 1
    if device.type != "cuda":
        return True
    hbm = torch.cuda.get_device_properties(device).total_memory
    return 2 * n / w > hbm / 3


def _grad_ring_auto(args, model, dp_group, offload_params: bool) -> int:
    """--offload-grad-ring auto.  The ring (4 unit-sized pinned slots instead of a whole-model host
    gradient shard) measured (profiles/r4/s23, chapter 05 8B b1 x 4096, same box): with the
    parameter shard resident in HBM 16-30 % FASTER (the D2H of each unit's gradient and its host
    AdamW pipeline through the slots), with parameters on the host 3-5 % slower (the host thread
    waits for a slot behind the host updates).  So: on for the resident layout; with parameters
    on the host only when this node's ranks would not fit their whole host state in RAM
    (8 B per shard parameter -- bf16 parameters, gradients, m, v -- times the ranks on the node,
    against 85 % of MemAvailable), which is the 405B-on-one-node case.  Off under gradient
    accumulation (the ring has no whole-model shard to accumulate into)."""
    if max(1, args.grad_accum) != 1:
        return 0
    if not offload_params:
        return 4
    n = sum(p.numel() for p in model.parameters())
    w = torch.distributed.get_world_size(dp_group) if torch.distributed.is_initialized() else 1
    local = int(os.environ.get("LOCAL_WORLD_SIZE", "1") or 1)
    try:
        import psutil

        avail = psutil.virtual_memory().available
    except Exception:  # pragma: no cover - psutil is in the image
        return 4
    need = 8 * (n / max(1, w)) * max(1, local)
    return 4 if need > 0.85 * avail else 0


def _scheduler(args, opt):
    if getattr(args, "ds_scheduler", None) and args.ds_scheduler.get("type") == "WarmupCosineLR":
        p = args.ds_scheduler.get("params", {})
        total = int(p.get("total_num_steps", 1000))
        warm = int(p.get("warmup_num_steps", 0))
        floor = float(p.get("cos_min_ratio", 1e-2))

        def f(step):
            if step < warm:
                return (step + 1) / max(1, warm)
            t = min(1.0, (step - warm) / max(1, total - warm))
            return floor + (1 - floor) * 0.5 * (1 + math.cos(math.pi * t))

        return torch.optim.lr_scheduler.LambdaLR(opt, f)
    # reference: CosineAnnealingLR(T_max=1000, eta_min=lr*1e-2), stepped every optimizer step
    return torch.optim.lr_scheduler.CosineAnnealingLR(opt, T_max=1000, eta_min=args.lr * 1e-2)


def xgmi_timeout(flag) -> float:
    """xGMI barrier timeout: an explicit --tp-comm-timeout wins over DTG_XGMI_TIMEOUT (logged
    when they disagree), which wins over the 60 s default."""
    env = os.environ.get("DTG_XGMI_TIMEOUT")
    if flag is not None:
        if env is not None and float(env) != float(flag):
            LOGGER.warning(f"--tp-comm-timeout {flag:g} overrides DTG_XGMI_TIMEOUT={env}")
        return float(flag)
    return float(env) if env is not None else 60.0


def _resolve_dp_comm(args, chapter, cfg, device, dp_group, world, fsdp, pp, nseq) -> str:
    """--dp-comm auto: RCCL vs the copy-engine path, timed on the data-parallel group at this
    job's message size (ZeRO: one gradient bucket; FSDP: one decoder layer's flat parameters).
    Only ZeRO and FSDP have a copy-engine path; everything else is RCCL without measuring."""
    zero = chapter == "02" and getattr(args, "dp_mode", "zero") == "zero" and pp == 1 and nseq == 1
    forced = bool(os.environ.get("DTG_TRANSPORT_CHILD_CMD"))  # tests: the child path on CPU
    if (device.type != "cuda" and not forced) or world == 1 or not (zero or fsdp) or \
            getattr(args, "cpu_offload", "off") == "on":
        return "rccl"
    from ..parallel import transport

    if zero:  # one gradient bucket (a model smaller than a bucket is one bucket)
        msg = min(args.bucket_mb << 20, 2 * cfg.num_params())
    else:
        tp = max(1, getattr(args, "tp", 1)) if chapter == "07" else 1
        emb = cfg.vocab_size * cfg.hidden_size * (1 if getattr(cfg, "tie_word_embeddings", False) else 2)
        msg = 2 * ((cfg.num_params() - emb) // max(1, cfg.num_hidden_layers)) // tp
    if chapter == "07":
        mesh = (max(1, getattr(args, "tp", 1)), 0)
    elif getattr(args, "sharding", "full") == "hybrid":
        mesh = (args.shard_size or int(os.environ.get("LOCAL_WORLD_SIZE", torch.cuda.device_count() or 1)), 1)
    else:
        mesh = (1, 0)
    choice, args.dp_comm_calibration = transport.resolve_isolated("auto", "dp", device, msg, mesh=mesh, log=LOGGER.info)
    return choice


def _build(args, chapter, device, world):
    """Model + engine + optimizer for a chapter.  Returns (model, engine, dp_size, dp_rank, ckpt_style)."""
    depth = getattr(args, "num_layers", None)
    cfg = resolve_config(args.model_name, **({} if depth is None else {"num_hidden_layers": depth}))
    if chapter == "rime" and cfg.vocab_size != 156939:
        LOGGER.warning("rime chapter expects the +28,683-token vocabulary (llama-3.2-3b-rime)")
    tp_group = dp_group = None
    dp_size, dp_rank = world, udist.get_rank()
    if chapter in ("06", "07"):
        from ..parallel.tensor_parallel import make_mesh

        tp = args.tp if chapter == "07" else int(os.environ.get("LOCAL_WORLD_SIZE", torch.cuda.device_count() or 1))
        tp = max(1, min(tp, world))
        dp_group, tp_group, dp_rank, tp_rank, dp_size = make_mesh(tp)
        LOGGER.info(f"mesh: dp={dp_size} tp={tp} (dp_rank={dp_rank}, tp_rank={tp_rank})")
        if getattr(args, "tp_comm", "rccl") == "auto" and tp_group is not None:
            from ..parallel import transport

            chunks = max(1, getattr(args, "tp_overlap_chunks", 2))
            msg = transport.tp_message_bytes(args.batch_size, args.seq_length, cfg.hidden_size) // chunks
            args.tp_comm, args.tp_comm_calibration = transport.resolve_isolated(
                "auto", "tp", device, msg, mesh=(tp, 1), timeout_s=xgmi_timeout(getattr(args, "tp_comm_timeout", None)),
                log=LOGGER.info)
        if getattr(args, "tp_comm", "rccl").startswith("xgmi") and tp_group is not None and device.type == "cuda":
            from ..parallel.xgmi import XgmiCommunicator
            from ..utils import comm as _comm

            engine = "dma" if args.tp_comm == "xgmi-dma" else "kernel"
            timeout = xgmi_timeout(getattr(args, "tp_comm_timeout", None))
            _comm.register_xgmi(tp_group, XgmiCommunicator(tp_group, capacity_bytes=args.tp_comm_mb << 20, device=device,
                                                           gather_engine=engine, timeout_s=timeout))
            LOGGER.info(f"tp collectives: direct-peer xGMI ({args.tp_comm_mb} MiB workspace per rank, "
                        f"collectives on {'copy engines' if engine == 'dma' else 'pull kernels'}, barrier timeout {timeout:g} s)")
    seq = None  # (kind, group, rank, degree): Ulysses / context parallel over each row
    nseq = max(getattr(args, "sp", 1), getattr(args, "cp", 1))
    if nseq > 1:
        assert min(getattr(args, "sp", 1), getattr(args, "cp", 1)) == 1, "--sp and --cp are alternatives"
        from ..parallel.tensor_parallel import make_mesh

        dp_group, seq_group, dp_rank, seq_rank, dp_size = make_mesh(nseq)
        seq = ("sp" if args.sp > 1 else "cp", seq_group, seq_rank, nseq)
        LOGGER.info(f"mesh: dp={dp_size} x {seq[0]}={nseq} (dp_rank={dp_rank}, {seq[0]}_rank={seq_rank})")
    pp = max(1, getattr(args, "pp", 1))
    pp_group = None
    if pp > 1:
        assert nseq == 1, "--pp is not combined with --sp / --cp"
        from ..parallel.tensor_parallel import make_mesh

        # contiguous ranks form one pipeline (its P-1 boundaries on distinct xGMI links);
        # strided groups are the data-parallel replicas of each stage
        dp_group, pp_group, dp_rank, pp_rank, dp_size = make_mesh(pp)
        LOGGER.info(f"mesh: dp={dp_size} x pp={pp} (dp_rank={dp_rank}, stage={pp_rank})")
    replicate_group = None
    if getattr(args, "sharding", "full") == "hybrid" and world > 1:
        from ..parallel.tensor_parallel import make_mesh

        shard = args.shard_size or int(os.environ.get("LOCAL_WORLD_SIZE", torch.cuda.device_count() or 1))
        shard = max(1, min(shard, world))
        # contiguous groups of `shard` ranks hold one sharded replica; strided groups replicate
        replicate_group, dp_group, _, _, n_rep = make_mesh(shard)
        LOGGER.info(f"hybrid sharding: {n_rep} replicas x {shard}-way shards")
    fsdp = chapter in ("04", "05", "07") or (chapter == "deepspeed" and args.zero_stage == 3)
    if getattr(args, "dp_comm", "rccl") == "auto":
        args.dp_comm = _resolve_dp_comm(args, chapter, cfg, device, dp_group, world, fsdp, pp, nseq)
    if fsdp:
        with torch.device("meta"):
            model = build_model(cfg, tp_group=tp_group, init=False)
    elif seq is not None:
        model = build_model(cfg, device=device, **{f"{seq[0]}_group": seq[1]})
    else:
        model = build_model(cfg, device=device, tp_group=tp_group)
    if tp_group is not None and hasattr(model, "tp"):
        model.tp.overlap_chunks = max(1, getattr(args, "tp_overlap_chunks", 2))
        LOGGER.info(f"tp overlap: {model.tp.overlap_chunks} chunks per sequence-parallel region")
        model.tp.sp_regather = getattr(args, "sp_regather", "off") == "on"
        if model.tp.sp_regather:
            LOGGER.info("sp regather: column-parallel inputs re-gathered in the backward (not kept)")
    model._dtg_seq = seq
    model._dtg_pp = None
    if pp > 1:
        from ..parallel.pipeline import PipelineStage

        stage = PipelineStage(model, pp_group)
        model._dtg_layer_offset = stage.layer_range[0]  # checkpoints use global layer names
        model._dtg_pp = stage
        LOGGER.info(f"pipeline stage {stage.stage}/{pp}: layers [{stage.layer_range[0]}, {stage.layer_range[1]})")
    model._dtg_ac_auto = None
    if args.activation_checkpointing == "on":
        spec = str(getattr(args, "ac_layers", "all"))
        apply_activation_checkpointing(model, count=None if spec in ("all", "auto") else int(spec))
        if spec == "auto":
            model._dtg_ac_auto = {"tp": tp_group.size() if tp_group is not None else 1,
                                  "regather": getattr(args, "sp_regather", "off") == "on"}
        LOGGER.info(f"activation checkpointing: {checkpointed_count(model)} of {len(model.layers)} layers"
                    + (" (auto: re-planned after step 1 against --ac-budget-gb)" if spec == "auto" else ""))
    LOGGER.info(f"{sum(p.numel() for p in model.parameters()) / 1e9:.3f}B parameters (this rank's shard of TP)")
    LOGGER.info(f"Before engine: {get_mem_stats(device)}")
    if fsdp:
        from ..parallel.fsdp import FullyShard

        policy = "size" if chapter == "04" else "transformer"
        cpu_offload = getattr(args, "cpu_offload", "off") == "on"
        offload_params = _offload_params(args, model, dp_group, device) if cpu_offload else True
        if cpu_offload:
            LOGGER.info("cpu offload: " + ("parameters, gradients and AdamW state on the host" if offload_params else
                                           "gradients and AdamW state on the host, parameter shard resident in HBM"))
        ring = str(getattr(args, "offload_grad_ring", "0"))
        if not cpu_offload:
            ring = 0
        elif ring == "auto":
            ring = _grad_ring_auto(args, model, dp_group, offload_params)
        else:
            ring = int(ring)
        if ring:
            LOGGER.info(f"cpu offload: host gradient ring of {ring} unit-sized pinned slots (no whole-model "
                        "host gradient shard)")
        engine = FullyShard(model, group=dp_group, tp_group=tp_group, policy=policy,
                            min_num_params=getattr(args, "numel_to_wrap", 100_000_000), device=device,
                            reshard_after_forward=args.reshard_after_forward == "on",
                            cpu_offload=cpu_offload, offload_params=offload_params, seed=args.seed,
                            replicate_group=replicate_group, grad_ring=ring,
                            dp_comm=getattr(args, "dp_comm", "rccl") if device.type == "cuda" else "rccl")
        if getattr(engine, "xdp", None) is not None:
            LOGGER.info("FSDP collectives: copy-engine pulls over xGMI (shared shard buffers, gradient pool)")
        style = "sharded"
    else:
        if world == 1 or (pp > 1 and dp_size == 1):
            mode = "single"
        elif pp > 1:
            mode = args.dp_mode if chapter == "02" else "ddp"
        elif seq is not None:  # parameters replicated on every rank; the row's loss is split over seq ranks
            mode = args.dp_mode if chapter == "02" else "ddp"
        elif chapter in ("01", "rime"):
            mode = "single"
        elif chapter == "02":
            mode = args.dp_mode
        elif chapter == "deepspeed":
            mode = "ddp" if args.zero_stage == 0 else "zero"
        else:  # 06: data parallel across TP groups
            mode = "ddp"
        engine = DataParallel(model, mode=mode, group=dp_group if pp > 1 else (None if seq is not None else dp_group),
                              tp_group=tp_group,
                              bucket_mb=args.bucket_mb, broadcast_from_rank0=tp_group is None,
                              grad_divisor=dp_size if seq is not None else None,
                              dp_comm=getattr(args, "dp_comm", "rccl") if device.type == "cuda" else "rccl")
        if getattr(engine, "xdp", None) is not None:
            LOGGER.info("ZeRO collectives: copy-engine pulls over xGMI between the ranks' shared flat buffers")
        style = "full" if mode == "single" and chapter in ("01", "rime") else ("dp" if chapter == "02" else "sharded")
        if pp > 1:
            style = "sharded"  # no rank holds the whole model: no model.pt
    if model._dtg_pp is not None:
        from ..parallel.pipeline import OneFOneB

        assert max(1, args.grad_accum) == 1, "--pp: the pipeline's micro-batches are the accumulation (--pp-microbatches)"
        model._dtg_pp = OneFOneB(model._dtg_pp, engine, num_microbatches=args.pp_microbatches)
    LOGGER.info(f"After engine ({engine.mode}): {get_mem_stats(device)}")
    if args.init_from:
        from ..models.loading import load_pretrained

        load_pretrained(engine, args.init_from, cfg)
    return model, engine, dp_size, dp_rank, style, cfg


def run(chapter: str, argv=None):
    parser = get_parser(chapter)
    args = parser.parse_args(argv)
    if chapter == "deepspeed":
        args = _deepspeed_overrides(args)
    rank, local_rank, world, device = udist.init_distributed(local_rank_arg=getattr(args, "local_rank", None))
    if getattr(args, "detect_anomaly", "off") == "on":
        torch.autograd.set_detect_anomaly(True, check_nan=True)
    udist.setup_logging(rank, with_rank=chapter not in ("01", "rime"))
    LOGGER.info(os.environ)
    LOGGER.info(args)
    LOGGER.info(f"local_rank={local_rank} rank={rank} world size={world}")
    # host CPU share and NUMA placement of this rank (chapter 05's offload is host-bound)
    LOGGER.info(f"host placement: {udist.host_placement(device, pin=getattr(args, 'pin_numa', 'off') == 'on', share=getattr(args, 'cpu_share', 0))}")
    if args.tunableop != "off" and device.type == "cuda":
        from ..utils.gemm_tuning import enable_tunableop

        enable_tunableop(tune=args.tunableop == "tune")
    random.seed(args.seed)
    torch.manual_seed(args.seed)
    if args.determinism == "on":
        torch.use_deterministic_algorithms(True, warn_only=True)

    model, engine, dp_size, dp_rank, style, cfg = _build(args, chapter, device, world)
    opt = FlatAdamW(engine, lr=args.lr, betas=getattr(args, "betas", (0.9, 0.999)), eps=getattr(args, "eps", 1e-8),
                    weight_decay=getattr(args, "weight_decay", 0.01))
    lr_scheduler = _scheduler(args, opt)

    # ---- data (reference E1-E8); synthetic by default on the offline boxes
    with udist.rank0_first():
        eos = getattr(cfg, "eos_token_id", None)
        train_data, seq_length, collate = dtg_data.build_dataset(
            args.dataset_name, tokenizer_name=args.model_name, seq_length=args.seq_length,
            vocab_size=cfg.vocab_size, max_position_embeddings=cfg.max_position_embeddings,
            num_samples=args.num_samples, eos_id=eos, seed=args.seed)
    LOGGER.info(f"{len(train_data)} training samples, seq_length={seq_length}")
    dataloader = dtg_data.build_dataloader(train_data, args.batch_size, collate, dp_size=dp_size, dp_rank=dp_rank,
                                           shuffle=chapter != "rime", num_workers=args.num_workers,
                                           prefetch_factor=args.prefetch_factor, seed=args.seed)
    LOGGER.info(f"{len(dataloader)} batches per epoch")

    exp_dir = Path(args.save_dir) / args.experiment_name
    state = new_state()
    resumed = False
    fmt = getattr(args, "ckpt_format", "dcp")
    mgr = CheckpointManager(exp_dir, engine, opt, lr_scheduler, style, local_rank,
                            async_save=getattr(args, "async_ckpt", "off") == "on", fmt=fmt)
    # DTG_FAKE_WORLD rehearsal: the other ranks are a fake process group, so its weights are
    # not a training result -- never resume into it, never write (or journal-commit) a checkpoint
    fake = udist.fake_world() > 1
    if fake:
        if has_checkpoint(exp_dir) or (exp_dir / CheckpointManager.PENDING).exists():
            raise SystemExit(f"DTG_FAKE_WORLD rehearsal refuses to run in {exp_dir}: it holds a checkpoint "
                             "(a rehearsal's state is not a training result); use a fresh --experiment-name")
        LOGGER.warning("DTG_FAKE_WORLD rehearsal: checkpoint saving disabled")
    elif rank == 0 and exp_dir.exists():  # finish (or discard) a save interrupted by a crash
        how = recover_checkpoint(exp_dir)
        if how != "clean":
            LOGGER.warning(f"{exp_dir}: interrupted checkpoint save {how}")
    udist.barrier()
    if not fake and has_checkpoint(exp_dir):
        LOGGER.info(f"Resuming from {exp_dir}")
        t_load = time.perf_counter()
        state = mgr.load()
        LOGGER.info(f"checkpoint loaded in {time.perf_counter() - t_load:.2f} s")
        resumed = True
    LOGGER.info(f"Resumed={resumed} | {state}")
    udist.make_exp_dir(exp_dir, per_rank_dirs=chapter in ("04", "deepspeed"))
    wb_kw = wandb_init_kwargs(getattr(args, "wandb_mode", "rank0"), exp_dir, args.experiment_name, rank, local_rank,
                              resumed, config={"args": vars(args), "training_data_size": len(train_data),
                                               "num_batches": len(dataloader), "world_size": world})
    sink = MetricSink(exp_dir, rank, use_wandb=args.wandb != "off", wandb_kwargs=wb_kw)

    waiting = getattr(args, "waiting_timers", "off") == "on" and world > 1
    names = ("data", "forward", "backward", "update") + (("waiting",) if waiting else ())
    timers = make_timers(device, names=names, sync=args.sync_timers == "on", ranges=args.roctx == "on")
    prof = None
    prof_start, prof_stop = 3, 3 + args.torch_profile_steps

    def wait_for_peers():
        # Straggler probe (related-topics/optimizing-data-loading): time spent in a barrier
        # before each phase is time this rank waited for the slowest one.
        if waiting:
            with timers["waiting"]:
                torch.distributed.barrier()
    tok_per_step = dp_size * args.batch_size * seq_length * max(1, args.grad_accum)
    flops_tok = cfg.flops_per_token(seq_length)
    mem_suffix = "_in_gb" if chapter in ("05", "deepspeed") else "_gb"
    fault_rng = random.Random(args.seed * 1000 + rank + 7 * state["global_step"])
    accum = max(1, args.grad_accum)
    seq_shard = _seq_sharder(model._dtg_seq)
    model.train()
    graphed = None
    if getattr(args, "hip_graph", "off") == "on":
        if device.type == "cuda" and getattr(engine, "mode", None) == "single" and accum == 1:
            from .graph import GraphedStep

            graphed = GraphedStep(model, engine, opt, scheduler=None, warmup=3)
            LOGGER.info("HIP graph: the training step is captured after 3 eager steps and replayed "
                        "(time/forward covers the whole step; time/backward and time/update read 0)")
        else:
            LOGGER.warning("--hip-graph needs one GPU, a single-process engine and --grad-accum 1; running eagerly")
    run_loss = None  # device-side running-loss accumulator (flushed into state at log / ckpt steps)
    for state["epoch"] in range(state["epoch"], args.num_epochs):
        LOGGER.info(f"Begin epoch {state['epoch']} at step {state['epoch_step']}")
        sampler = dataloader.sampler
        # every chapter sets the epoch (06/07 forgot it: SURVEY §2.11 #3); a resumed epoch starts
        # at its first unconsumed sample instead of re-reading the consumed batches
        per_step = args.batch_size * accum
        sampler.set_epoch(state["epoch"], skip=state["epoch_step"] * per_step)
        batches = iter(dataloader)
        n_steps = (sampler.full_len() // args.batch_size) // accum
        # progress bar: rank 0 only, resumable; chapters 05-07 keep it off as the
        # reference does (their logs are per-rank files)
        progress = tqdm(total=n_steps, initial=state["epoch_step"], dynamic_ncols=True,
                        disable=rank > 0 or chapter in ("05", "06", "07"))
        for i_step in range(state["epoch_step"], n_steps):
            progress.update(1)
            micro = []
            with timers["data"], torch.no_grad():
                for _ in range(accum):
                    b = next(batches)
                    nv = b.pop("num_valid", None)
                    if nv is None:
                        nv = count_valid_labels(b["labels"])
                    mx = b.pop("max_seqlen", None)
                    b = {k: v.to(device=device, non_blocking=True) for k, v in b.items()}
                    b["num_valid"] = nv
                    if seq_shard is not None:
                        b = seq_shard(b)
                    if mx is not None:
                        b["max_seqlen"] = mx
                    micro.append(b)
            if args.fault_inject_prob > 0 and fault_rng.random() < args.fault_inject_prob:
                raise RuntimeError(f"injected fault at global step {state['global_step']} on rank {rank}")
            if graphed is not None and "position_ids" not in micro[0]:
                b = dict(micro[0])
                nv = b.pop("num_valid")
                b.pop("max_seqlen", None)
                with timers["forward"]:
                    loss_sum = graphed(b, num_valid=nv).detach()
                with timers["update"]:
                    lr_scheduler.step()
                micro = []
            else:
                opt.zero_grad(set_to_none=True)
                loss_sum = None
            if model._dtg_pp is not None and micro:  # 1F1B: forward and backward interleaved
                b = micro[0]
                wait_for_peers()
                with timers["forward"]:
                    loss_sum = model._dtg_pp.step(b["input_ids"], labels=b["labels"], num_valid=b["num_valid"],
                                                  position_ids=b.get("position_ids")).detach()
                micro_pp, micro = micro, []
            for j, b in enumerate(micro):
                ctx = engine.no_sync() if j < accum - 1 else _null()
                with ctx:
                    wait_for_peers()
                    with timers["forward"]:
                        out = model(**b)
                    wait_for_peers()
                    with timers["backward"]:
                        engine.backward(out.loss)
                loss_sum = out.loss.detach() if loss_sum is None else loss_sum + out.loss.detach()
            if model._dtg_pp is not None:
                micro = micro_pp
            check = getattr(args, "check_finite", "off")
            if check in ("on", "grad"):
                _report_nonfinite(model, engine, loss_sum, state["global_step"] + 1, rank, "grad")
            if micro:
                wait_for_peers()
                with timers["update"]:
                    opt.step()
                    lr_scheduler.step()
                if check in ("on", "param"):
                    _report_nonfinite(model, engine, None, state["global_step"] + 1, rank, "param")
            if seq_shard is not None:  # each sequence rank holds its share of the row losses
                loss_sum = loss_sum.clone()
                torch.distributed.all_reduce(loss_sum, group=model._dtg_seq[1])
            state["global_step"] += 1
            state["epoch_step"] += 1
            if model._dtg_ac_auto is not None and _plan_ac_layers(args, model, cfg, device, model._dtg_ac_auto,
                                                                  seq_length):
                model._dtg_ac_auto = None
            # host read of the xGMI communicators' pinned error words (no device sync): a peer
            # lost in this step's barriers stops the job here, not at the next log step
            ucomm.poll_xgmi()
            if args.torch_profile_steps > 0:
                prof = _profile_tick(prof, state["global_step"], prof_start, prof_stop, exp_dir, rank, device)
            # summed on the device; one host sync per --log-freq window / checkpoint instead of the
            # reference's `.item()` every step
            run_loss = loss_sum / accum if run_loss is None else run_loss + loss_sum / accum

            if state["global_step"] % args.log_freq == 0 or state["global_step"] % args.ckpt_freq == 0:
                state["running_loss"] += float(run_loss.item())
                run_loss = None
            if state["global_step"] % args.log_freq == 0:
                ucomm.check_xgmi()  # a timed-out xGMI barrier ends the job here (non-zero exit)
                ms_per_step = sum(t.avg_elapsed_ms() for t in timers.values())
                tps = 1000 * tok_per_step / ms_per_step if ms_per_step > 0 else 0.0
                info = {
                    "global_step": state["global_step"],
                    "lr": lr_scheduler.get_last_lr()[0],
                    "running_loss": state["running_loss"] / args.log_freq,
                    "epoch": state["epoch"],
                    "epoch_progress": state["epoch_step"] / n_steps,
                    "num_batches_remaining": n_steps - i_step,
                    **get_mem_stats(device, mem_suffix),
                    "tok/s": tps,
                    "tok/s/gpu": tps / world,
                    "mfu": tps * flops_tok / (world * MI355X_BF16_DENSE_FLOPS) if device.type == "cuda" else 0.0,
                    "time/total": ms_per_step,
                    **{f"time/{k}": t.avg_elapsed_ms() for k, t in timers.items()},
                }
                if getattr(engine, "cpu_offload", False):
                    info.update(_offload_info(engine))
                if args.activation_checkpointing == "on":
                    info["ac/layers"] = checkpointed_count(model)
                LOGGER.info(info)
                sink.log(info, state["global_step"])
                if device.type == "cuda":
                    torch.cuda.reset_peak_memory_stats(device)
                state["running_loss"] = 0
                for t in timers.values():
                    t.reset()

            if state["global_step"] % args.ckpt_freq == 0 and not fake:
                ucomm.check_xgmi()  # never checkpoint state computed from stale peer data
                LOGGER.info("Saving checkpoint.")
                t_save = time.perf_counter()
                mgr.save(state)
                LOGGER.info(f"checkpoint save: training stalled {time.perf_counter() - t_save:.2f} s"
                            + (" (async: snapshot only; the files are written in the background)" if mgr.async_save else ""))
            if args.max_steps and state["global_step"] >= args.max_steps:
                if run_loss is not None:
                    state["running_loss"] += float(run_loss.item())
                LOGGER.info(f"Reached --max-steps {args.max_steps}")
                progress.close()
                t_fin = time.perf_counter()
                mgr.finalize()
                if mgr.async_save:
                    LOGGER.info(f"checkpoint finalize (join the writer, publish): {time.perf_counter() - t_fin:.2f} s")
                ucomm.check_xgmi()
                return state
        progress.close()
        state["epoch_step"] = 0
    if run_loss is not None:
        state["running_loss"] += float(run_loss.item())
    mgr.finalize()
    ucomm.check_xgmi()
    return state


def _agree_max(value: int, device) -> int:
    """The largest value any rank holds (every rank calls it)."""
    import torch.distributed as dist

    if dist.is_initialized() and dist.get_world_size() > 1:
        t = torch.tensor([int(value)], dtype=torch.int64, device=device if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return int(t.item())
    return int(value)


def _plan_ac_layers(args, model, cfg, device, plan: dict, seq_length: int, peak_bytes=None) -> bool:
    """--ac-layers auto: keep checkpointed only as many layers as the HBM budget requires.
    Measured, over the first steps:
      1. after step 1 (every layer checkpointed) the step's peak P1 is read, and layers are
         released by the analytical per-layer size (layer_activation_bytes, x1.5);
      2. after step 2 the peak with those layers released gives the MEASURED cost of a released
         layer, (P2 - P1) / released, and the count is re-planned from P1 with it (x1.05);
      3. after steps 3 and 4, while the peak is still over the budget, the same re-plan from the
         larger release (a peak dominated by a transient at small releases -- the loss head, a
         gathered FSDP unit -- hides part of the per-layer cost at step 2: the 405B FSDP rank
         measured 1.04 GB per layer there and overshot at 73 released).
    Peaks are the caching allocator's reserved bytes (what the HBM really holds), reset at each
    planning step.  Every rank takes the largest count any rank needs (a recompute re-issues the
    layer's TP collectives).  `plan` carries the state between calls; returns True when done."""
    from ..parallel.checkpointing import ac_layers_for_budget, layer_activation_bytes, set_checkpointed_layers

    n = len(model.layers)
    if peak_bytes is None:
        if device.type != "cuda":
            LOGGER.info("--ac-layers auto: no HBM to plan against off the GPU; every layer stays checkpointed")
            return True
        peak_bytes = torch.cuda.max_memory_reserved(device)
    budget = int(args.ac_budget_gb * 1e9)
    est = layer_activation_bytes(cfg, args.batch_size, seq_length, plan["tp"], plan.get("regather", False))
    phase = plan.get("phase", 1)
    if phase == 1:
        n_ckpt = checkpointed_count(model)
        inp = 2 * cfg.hidden_size * args.batch_size * seq_length // max(1, plan["tp"])
        keep = _agree_max(ac_layers_for_budget(n, n_ckpt, int(peak_bytes), budget, est, inp, safety=1.5), device)
        plan.update(p1=int(peak_bytes), released=n_ckpt - keep, phase=2)
        msg = f"step-1 peak {peak_bytes / 1e9:.1f} GB, ~{est / 1e9:.2f} GB per released layer (estimate)"
        done = plan["released"] == 0
    else:
        p1, released = plan["p1"], plan["released"]
        # never below a quarter of the estimate: a peak that did not grow (a reset peak counter,
        # an allocator that freed a cache) must not release every layer
        slope = max(1, est // 4, (int(peak_bytes) - p1) // max(1, released))
        over = int(peak_bytes) > budget
        if phase == 2 or over:
            keep = _agree_max(ac_layers_for_budget(n, n, p1, budget, slope, 0, safety=1.05), device)
            keep = max(keep, n - released) if phase > 2 else keep  # later steps only re-checkpoint
        else:
            keep = n - released
        plan.update(released=n - keep, phase=phase + 1)
        msg = (f"step-{phase} peak {peak_bytes / 1e9:.1f} GB with {released} layers released -> measured "
               f"{slope / 1e9:.2f} GB per released layer")
        done = (phase >= 2 and not over and phase > 2) or phase >= 4 or (phase == 2 and keep == n)
    changed = keep != checkpointed_count(model)
    set_checkpointed_layers(model, keep)
    if device.type == "cuda":
        if changed:  # hand back the blocks of the trial (re-reserving costs a step's worth of seconds)
            torch.cuda.empty_cache()
        torch.cuda.reset_peak_memory_stats(device)  # the next step's peak, not the trial's
    LOGGER.info(f"--ac-layers auto ({phase}): {msg}, budget {args.ac_budget_gb:g} GB -> {keep} of {n} layers "
                f"checkpointed" + ("" if done else "; checked again after the next step"))
    return done


def _offload_info(engine) -> dict:
    """CPU-offload record of the log window: host AdamW time and bandwidth, gradient D2H and
    parameter H2D volume and bandwidth per step (FullyShard.offload_stats), and this process's
    host memory: resident set, pinned shard buffers, and the host's MemAvailable."""
    out = {f"offload/{k}": v for k, v in engine.offload_stats().items()}
    bufs = [engine.shard_params, engine.shard_grads] + list(getattr(engine, "_ring", []))
    pinned = sum(t.numel() * t.element_size() for t in bufs if t.numel() and t.is_pinned())
    out["host/pinned_gb"] = pinned / 1e9
    try:
        import psutil

        out["host/rss_gb"] = psutil.Process().memory_info().rss / 1e9
        out["host/mem_available_gb"] = psutil.virtual_memory().available / 1e9
    except Exception:
        pass
    return out


def _report_nonfinite(model, engine, loss, step, rank, what):
    """--check-finite: name the parameters whose gradient (what="grad", after backward) or value
    (what="param", after the update) holds NaN/inf.  A ZeRO engine owns only its reduced gradient
    shard (the rest of the flat gradient buffer is scratch), so that shard is what is checked."""
    bad = []
    shard = getattr(engine, "grad_shard", None) if what == "grad" and getattr(engine, "mode", "") == "zero" else None
    if shard is not None:
        if not bool(torch.isfinite(shard).all()):
            bad.append(f"<ZeRO gradient shard: {int((~torch.isfinite(shard)).sum())} of {shard.numel()} elements>")
    else:
        for n, p in model.named_parameters():
            g = (p.grad if getattr(p, "main_grad", None) is None else p.main_grad) if what == "grad" else p.detach()
            if g is None or g.numel() == 0 or g.untyped_storage().size() == 0:  # e.g. a freed FSDP view
                continue
            if not bool(torch.isfinite(g).all()):
                bad.append(n)
    lf = loss is None or bool(torch.isfinite(loss).all())
    if bad or not lf:
        LOGGER.warning(f"[check-finite] step {step} rank {rank}: loss finite={lf}; non-finite {what} in "
                       f"{len(bad)} tensors: {bad[:12]}")


def _seq_sharder(seq):
    """Batch transform for --sp / --cp: this rank's slice of every row, labels shifted on the full
    rows, the global label count."""
    if seq is None:
        return None
    kind, _, r, n = seq

    def shard(b):
        if kind == "sp":
            from ..parallel.ulysses import ulysses_batch

            ids, lab, pos, nv = ulysses_batch(b["input_ids"], r, n, b.get("position_ids"), labels=b.get("labels"))
        else:
            from ..parallel.context_parallel import cp_batch

            ids, lab, pos, nv = cp_batch(b["input_ids"], r, n, labels=b.get("labels"), position_ids=b.get("position_ids"))
        out = {"input_ids": ids, "labels": lab, "num_valid": nv}
        if kind == "cp" and "cu_seqlens" in b:  # packed rows: the full rows' document boundaries
            out["cu_seqlens"] = b["cu_seqlens"]
        if pos is not None:
            out["position_ids"] = pos
        return out

    return shard


def _profile_tick(prof, step, start, stop, exp_dir, rank, device):
    """torch.profiler (ROCm kineto) over steps [start, stop): chrome trace per rank."""
    if step == start and prof is None:
        from torch.profiler import ProfilerActivity, profile

        acts = [ProfilerActivity.CPU] + ([ProfilerActivity.CUDA] if device.type == "cuda" else [])
        prof = profile(activities=acts, record_shapes=True)
        prof.__enter__()
    elif step == stop and prof is not None:
        prof.__exit__(None, None, None)
        path = Path(exp_dir) / f"trace-rank{rank}.json"
        prof.export_chrome_trace(str(path))
        LOGGER.info(f"torch.profiler trace written to {path}")
        prof = None
    return prof


class _null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def main(chapter: str, argv=None):
    """Entry point of every chapter's train_llm.py: @record error capture and a clean
    process-group teardown."""
    import faulthandler
    import signal

    try:  # `kill -USR1 <pid>` dumps every thread's Python stack (diagnosing-errors/README.md)
        faulthandler.register(signal.SIGUSR1, all_threads=True)
    except (AttributeError, ValueError):
        pass

    @udist.record
    def _main():
        try:
            return run(chapter, argv)
        finally:
            import torch.distributed as dist

            if dist.is_initialized():
                dist.destroy_process_group()

    return _main()
