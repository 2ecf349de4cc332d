"""Per-chapter command lines.

Flags, short forms and defaults are the reference's for every chapter; MI355X-specific knobs are
additive and never change a reference default.  Fixes: chapters 06/07 default `--seq-length` to
1024 instead of None, 07 accepts `--tp 1` (#4).
"""
import argparse

CHAPTERS = ("rime", "01", "02", "04", "05", "06", "07", "deepspeed")


def get_parser(chapter: str) -> argparse.ArgumentParser:
    assert chapter in CHAPTERS, chapter
    p = argparse.ArgumentParser(description=f"dtg chapter {chapter} causal-LM trainer (MI355X)")
    p.add_argument("-e", "--experiment-name", default=None, required=True)
    if chapter == "rime":
        p.add_argument("-d", "--dataset-name", default="synthetic:packed",
                       help="packed 8192-token rows: `disk:<path>` (datasets.load_from_disk) or synthetic:packed")
        p.add_argument("-m", "--model-name", default="llama-3.2-3b-rime")
    else:
        p.add_argument("-d", "--dataset-name", default=None, required=True,
                       help="HF dataset name/path, or `synthetic` / `synthetic:packed[:mean_doc_len]` / `synthetic:pattern` (learnable; offline)")
        p.add_argument("-m", "--model-name", default=None, required=True,
                       help="HF hub name (bundled configs: see dtg.models.available_configs) or config.json path")
    p.add_argument("--save-dir", default="../outputs")
    p.add_argument("--seed", default=0, type=int)
    p.add_argument("--num-epochs", default=1 if chapter == "rime" else 100, type=int)
    p.add_argument("--lr", default=3e-5, type=float)
    if chapter != "deepspeed":
        p.add_argument("-b", "--batch-size", default=1, type=int)
    p.add_argument("--log-freq", default=50 if chapter == "rime" else 100, type=int)
    p.add_argument("--ckpt-freq", default=500, type=int)
    p.add_argument("-s", "--seq-length", default=8192 if chapter == "rime" else 1024, type=int)
    if chapter == "04":
        p.add_argument("--numel-to-wrap", default=100_000_000, type=int,
                       help="Only applies FSDP to modules with numel > this value.")
    if chapter in ("04", "05", "07"):
        # 07: the 2-D recipe (FSDP over dp x TP over tp) with the 405B offload of chapter 05, so Llama-3.1-405B
        # fits ONE 8-GPU node (a TP-local 1/8 shard is 406 GB of bf16 state per rank without it)
        p.add_argument("--cpu-offload", default="on" if chapter == "05" else "off", choices=["on", "off"])
    if chapter in ("04", "05"):
        p.add_argument("--sharding", default="full", choices=["full", "hybrid"],
                       help="full: FULL_SHARD over all ranks; hybrid: shard within --shard-size ranks (one node), "
                            "replicate across nodes (HYBRID_SHARD)")
        p.add_argument("--shard-size", default=None, type=int, help="ranks per shard group (default LOCAL_WORLD_SIZE)")
    if chapter in ("04", "05", "07"):
        p.add_argument("--offload-params", default="auto", choices=["auto", "on", "off"],
                       help="with --cpu-offload on: on = parameters on the host too (reference); off = parameter "
                            "shard resident in HBM, only gradients + AdamW state offloaded; auto = off when the "
                            "shard fits a third of HBM")
        p.add_argument("--offload-grad-ring", default="auto",
                       help="with --cpu-offload on: stage each unit's reduced gradient in one of N unit-sized "
                            "pinned host slots consumed by the overlapped host AdamW, instead of a host gradient "
                            "shard for the whole model (saves 2 B/param of host RAM: 101 GB per rank for 405B at "
                            "W = 8); auto = 4 slots with the HBM-resident parameter layout, and with parameters "
                            "on the host only when the node's host state would not fit in RAM (profiles/r4/s23); "
                            "off under gradient accumulation; 0 = off")
    if chapter == "07":
        p.add_argument("--tp", default=8, type=int)
    if chapter in ("06", "07"):
        p.add_argument("--tp-comm", default="rccl", choices=["auto", "rccl", "xgmi", "xgmi-dma"],
                       help="TP/SP all-gather / reduce-scatter / all-reduce: RCCL, or the direct-peer xGMI "
                            "library (csrc/comm/xgmi.hip; one node per TP group); xgmi-dma moves the "
                            "all-gathers and reduce-scatters on the copy engines, one stream per peer (no CU "
                            "time under the overlapped GEMMs); auto = whichever of the three is fastest at this "
                            "job's message size on the TP group, timed at startup in a child job on the same GPUs "
                            "(parallel/transport.py; RCCL if the child fails).  Default rccl: the direct-peer "
                            "paths have not yet been validated across devices")
        p.add_argument("--tp-comm-mb", default=256, type=int, help="xGMI workspace per rank (largest TP message)")
        p.add_argument("--tp-comm-timeout", default=None, type=float,
                       help="seconds an xGMI barrier waits for a peer before the collective fails (default: "
                            "DTG_XGMI_TIMEOUT, else 60; this flag wins over the variable); the job then exits "
                            "non-zero at the end of that step")
        p.add_argument("--tp-overlap-chunks", default=2, type=int,
                       help="row chunks of the overlapped sequence-parallel regions (parallel/async_tp.py): the "
                            "all-gather / reduce-scatter of one chunk runs under the GEMMs of the next; 1 = off")
        p.add_argument("--sp-regather", default="off", choices=["on", "off"],
                       help="layers that do not recompute keep only their sequence-parallel shard of each "
                            "column-parallel GEMM's input and re-gather it in the backward (one more all-gather "
                            "per sub-block, prefetched; (1 - 1/tp) of a [tokens, hidden] tensor less per sub-block "
                            "and layer) -- with --ac-layers auto, more layers skip their recompute")
    if chapter == "deepspeed":
        p.add_argument("--local_rank", type=int, default=None)
        p.add_argument("--deepspeed", action="store_true", help="accepted for launcher compatibility")
        p.add_argument("--deepspeed_config", default=None, help="ds_config.json (train_micro_batch_size_per_gpu, "
                       "optimizer.params, scheduler.params, zero_optimization.stage)")
    # ---- additive MI355X knobs
    g = p.add_argument_group("dtg (MI355X) options")
    g.add_argument("--waiting-timers", default="off", choices=["on", "off"],
                   help="time a barrier before forward/backward/update (straggler detection)")
    g.add_argument("--roctx", default="off", choices=["on", "off"], help="roctx ranges around the step phases")
    g.add_argument("--torch-profile-steps", default=0, type=int,
                   help="record N steps (after the first 3) with torch.profiler; chrome trace in the exp dir")
    g.add_argument("--sync-timers", default="on", choices=["on", "off"],
                   help="on: reference LocalTimer (device sync around every phase); off: HIP-event timers")
    if chapter in ("rime", "01", "02"):
        g.add_argument("--sp", default=1, type=int,
                       help="Ulysses sequence parallel degree: each row is split over this many ranks, "
                            "all-to-all seq<->heads around attention (packed rows supported)")
        g.add_argument("--cp", default=1, type=int,
                       help="context parallel degree: zig-zag row shards, all-gathered K/V, one varlen flash call "
                            "per layer (dense or packed rows)")
        g.add_argument("--pp", default=1, type=int,
                       help="pipeline parallel degree: contiguous ranks form a pipeline of decoder-layer stages "
                            "(1F1B schedule, point-to-point activations); the rest is data parallel")
        g.add_argument("--pp-microbatches", default=4, type=int,
                       help="1F1B micro-batches per step (must divide --batch-size)")
    g.add_argument("--grad-accum", default=1, type=int, help="micro-batches per optimizer step (no_sync)")
    g.add_argument("--detect-anomaly", default="off", choices=["on", "off"],
                   help="debugging: torch.autograd anomaly mode (raises at the first backward op whose output "
                        "is NaN, with the forward stack that created it); slow")
    g.add_argument("--check-finite", default="off", choices=["on", "off", "grad", "param"],
                   help="debugging: log the tensors holding NaN/inf -- gradients after every backward (grad), "
                        "parameters after every update (param) or both (on); each check syncs the device")
    g.add_argument("--bucket-mb", default=256, type=int, help="gradient bucket size for DDP/ZeRO")
    if chapter in ("02", "04", "05", "07"):
        g.add_argument("--dp-comm", default="rccl", choices=["auto", "rccl", "xgmi-dma"],
                       help="ZeRO / FSDP collectives: RCCL, or copy-engine pulls between the ranks' shared shard / "
                            "gradient buffers over xGMI (one node; no CU time under the overlapped compute); "
                            "auto = the faster of the two at this job's bucket / layer size, timed at startup in a "
                            "child job (RCCL if the child fails).  Default rccl, as for --tp-comm")
    if chapter == "02":
        g.add_argument("--dp-mode", default="zero", choices=["ddp", "zero"],
                       help="zero: sharded optimizer (reference's ZeroRedundancyOptimizer); ddp: replicated")
    g.add_argument("--activation-checkpointing", default="on" if chapter == "05" else "off", choices=["on", "off"])
    g.add_argument("--ac-layers", default="all",
                   help="with --activation-checkpointing on: how many decoder layers recompute their forward "
                        "(the first N of this rank's stack; the others keep their activations).  all = every "
                        "layer (the reference); N; auto = as few as --ac-budget-gb allows, planned from the measured "
                        "peaks of steps 1 and 2 (agreed over all ranks)")
    g.add_argument("--ac-budget-gb", default=280.0, type=float,
                   help="HBM budget (GB = 1e9 bytes per GPU, reserved by the caching allocator) --ac-layers auto "
                        "plans against; an MI355X holds 309 GB (288 GiB), the rest is left to RCCL / fragmentation")
    g.add_argument("--reshard-after-forward", default="on", choices=["on", "off"])
    g.add_argument("--num-workers", default=1, type=int)
    g.add_argument("--prefetch-factor", default=2, type=int)
    g.add_argument("--num-samples", default=100_000, type=int, help="synthetic dataset size")
    g.add_argument("--max-steps", default=0, type=int, help="stop after this many optimizer steps (0 = no limit)")
    g.add_argument("--fault-inject-prob", default=0.0, type=float, help="raise on a step with this probability (elastic tests)")
    g.add_argument("--wandb", default="auto", choices=["auto", "off"])
    g.add_argument("--wandb-mode", default="rank0", choices=["rank0", "local_rank0", "every_rank"],
                   help="wandb run layout: one run from rank 0; one per node grouped by experiment; one per rank "
                        "grouped (related-topics/wandb-configurations)")
    g.add_argument("--determinism", default="off", choices=["on", "off"])
    g.add_argument("--pin-numa", default="off", choices=["on", "off"],
                   help="restrict each rank's CPU affinity to its GPU's NUMA node (host AdamW / D2H locality); "
                        "the placement is logged at startup either way")
    g.add_argument("--cpu-share", default=0, type=int,
                   help="restrict this rank to N CPUs (after --pin-numa; the host AdamW's OpenMP team follows "
                        "OMP_NUM_THREADS): rehearse one rank's share of a node's cores on a bigger host; 0 = all")
    g.add_argument("--num-layers", default=None, type=int,
                   help="override the model's num_hidden_layers (exact-width, reduced-depth runs)")
    g.add_argument("--init-from", default=None, help="HF safetensors directory to load pretrained weights from")
    g.add_argument("--tunableop", default="use", choices=["off", "use", "tune"])
    g.add_argument("--ckpt-format", default="dcp", choices=["dcp", "dtg"],
                   help="checkpoint/ of the sharded chapters (02, 04-07): dcp = torch.distributed.checkpoint "
                        "written by every rank (the reference's tree, readable by dcp_to_torch_save; resumes on "
                        "any world size / TP degree); dtg = this framework's dtg-sharded-v2 (index.json + "
                        "shard_rNNNNN.pt).  Resume reads either")
    g.add_argument("--async-ckpt", default="off", choices=["on", "off"],
                   help="snapshot checkpoints to host memory (reused pinned buffers) and write them on a "
                        "background thread -- DCP over a dedicated gloo group, or dtg-sharded-v2; published "
                        "(state.json written last) at the next save or at the end of training")
    g.add_argument("--hip-graph", default="off", choices=["on", "off"],
                   help="single GPU: capture the whole step (fwd+bwd+AdamW) in a HIP graph and replay it "
                        "(launch-bound small models; dense fixed-shape batches)")
    return p
