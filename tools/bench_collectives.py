#!/usr/bin/env python3
"""Collective bandwidth over xGMI: all_reduce, all_gather,
reduce_scatter and all_to_all over message sizes, reported as algorithm and bus bandwidth
(nccl-tests conventions), so bucket sizes for DDP/ZeRO/FSDP can be chosen from measurements.
`--impl xgmi` runs all_reduce / all_gather / reduce_scatter on the direct-peer library
(csrc/comm/xgmi.hip) instead of RCCL, for the TP/SP message sizes; `--impl xgmi-dma` on its
copy-engine variants (one stream per peer).  `--zero-copy` places every input in the xGMI
workspace first (what a producer GEMM writing there achieves), so the stage copy is skipped:
run with and without it to price the staging.  `--shared-device`: every rank on cuda:0 with a
gloo group for the handle exchange (a protocol/arithmetic rehearsal on a 1-GPU box).

    torchrun --standalone --nproc-per-node 8 tools/bench_collectives.py --json > coll.jsonl
    torchrun --standalone --nproc-per-node 8 tools/bench_collectives.py --impl xgmi --max-mb 128
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist


def _sync(device):
    if device.type == "cuda":
        torch.cuda.synchronize()


def bench(op, nbytes, world, device, iters, warmup, xg=None, zero_copy=False):
    # gloo (CPU rehearsal) has no bf16 reductions: fp32 elements there, same byte count
    dt_ = torch.bfloat16 if device.type == "cuda" else torch.float32
    n = nbytes // (2 if dt_ == torch.bfloat16 else 4)
    x = torch.randn(n, device=device).to(dt_)
    if zero_copy and xg is not None:  # the input already lives in the workspace: no stage copy
        ws = xg.ws[:nbytes].view(dt_)
        ws.copy_(x)
        x = ws
    if op == "all_reduce":
        fn = (lambda: xg.all_reduce_(x)) if xg else (lambda: dist.all_reduce(x))
        factor = 2 * (world - 1) / world
    elif op == "all_gather":
        out = torch.empty(n * world, device=device, dtype=dt_)
        fn = (lambda: xg.all_gather_into(out, x)) if xg else (lambda: dist.all_gather_into_tensor(out, x))
        factor = (world - 1) / world
        nbytes = nbytes * world
    elif op == "reduce_scatter":
        out = torch.empty(n // world, device=device, dtype=dt_)
        fn = (lambda: xg.reduce_scatter_into(out, x)) if xg else (lambda: dist.reduce_scatter_tensor(out, x))
        factor = (world - 1) / world
    else:
        out = torch.empty_like(x)
        fn = lambda: dist.all_to_all_single(out, x)
        factor = (world - 1) / world
    for _ in range(warmup):
        fn()
    _sync(device)
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    _sync(device)
    dt = (time.perf_counter() - t0) / iters
    algbw = nbytes / dt / 1e9
    return dt * 1e6, algbw, algbw * factor


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ops", default="all_reduce,all_gather,reduce_scatter,all_to_all")
    ap.add_argument("--min-mb", type=float, default=1)
    ap.add_argument("--max-mb", type=float, default=1024)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--json", action="store_true")
    ap.add_argument("--impl", default="rccl", choices=["rccl", "xgmi", "xgmi-dma"])
    ap.add_argument("--zero-copy", action="store_true", help="xgmi: inputs pre-placed in the workspace")
    ap.add_argument("--shared-device", action="store_true", help="all ranks on cuda:0, gloo handle exchange")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo: CPU rehearsal of the harness (fp32 elements, no GPU)")
    a = ap.parse_args()
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.backend == "gloo":
        assert a.impl == "rccl", "--impl xgmi needs GPUs"
        device = torch.device("cpu")
        dist.init_process_group("gloo")
    elif a.shared_device:
        assert a.impl != "rccl", "--shared-device rehearses the xgmi library"
        device = torch.device("cuda", 0)
        torch.cuda.set_device(device)
        dist.init_process_group("gloo")
    else:
        device = torch.device("cuda", local)
        torch.cuda.set_device(device)
        dist.init_process_group("nccl", device_id=device)
    world, rank = dist.get_world_size(), dist.get_rank()
    xg = None
    ops = a.ops.split(",")
    if a.impl.startswith("xgmi"):
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
        import dtg  # noqa: F401
        from dtg.parallel.xgmi import XgmiCommunicator

        xg = XgmiCommunicator(None, capacity_bytes=int(a.max_mb * (1 << 20)) + (1 << 20), device=device,
                              gather_engine="dma" if a.impl == "xgmi-dma" else "kernel")
        ops = [o for o in ops if o != "all_to_all"]
    size = a.min_mb
    while size <= a.max_mb:
        nbytes = int(size * (1 << 20)) // (4 * world) * (4 * world)
        for op in ops:
            if a.zero_copy and op == "all_reduce":  # in place: the result cannot live in the workspace
                continue
            us, alg, bus = bench(op, nbytes, world, device, a.iters, a.warmup, xg, a.zero_copy)
            if rank == 0:
                rec = {"op": op, "impl": a.impl, "zero_copy": a.zero_copy, "shared_device": a.shared_device,
                       "bytes": nbytes, "world": world, "time_us": round(us, 1),
                       "algbw_GBps": round(alg, 2),
                       "busbw_GBps": round(bus, 2)}
                print(json.dumps(rec) if a.json else f"{op:15s} {nbytes / 2**20:9.1f} MiB {us:10.1f} us  "
                      f"algbw {alg:7.1f} GB/s  busbw {bus:7.1f} GB/s", flush=True)
        size *= 2
    if xg is not None:
        xg.check()
        xg.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main())
