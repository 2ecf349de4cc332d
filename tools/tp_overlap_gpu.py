#!/usr/bin/env python3
"""Tensor-parallel step with and without the overlapped SP regions (parallel/async_tp.py),
TP = 2 on ONE GPU: two ranks share the device, their sequence all-gathers / reduce-scatters run
through the direct-peer xGMI library (csrc/comm/xgmi.hip) on a side stream, and gloo only
exchanges the IPC handles.

    python tools/tp_overlap_gpu.py --chunks 1 4            # ms/step per chunk count
    rocprofv3 --kernel-trace -d gpurun_out/tp -o %pid%_run -- python3 tools/tp_overlap_gpu.py --chunks 4
    python tools/tp_overlap_gpu.py --trace gpurun_out/tp   # comm/compute overlap from the trace

With both ranks on one device the step time measures contention more than link speed; the
trace answers the question that transfers to an 8-GPU node: do the collective kernels run
concurrently with the GEMMs of the same rank (chunks > 1) or strictly between them (chunks = 1)?
The parent process never touches the GPU (ranks are spawned).
"""
import argparse
import csv
import glob
import json
import os
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)


def _worker(rank, world, port, chunks_list, layers, batch, seq, steps, outdir, engine="kernel"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import torch
    import torch.distributed as dist

    import dtg  # noqa: F401
    from dtg.models import build_model, resolve_config
    from dtg.parallel.data_parallel import DataParallel, FlatAdamW
    from dtg.parallel.tensor_parallel import make_mesh
    from dtg.parallel.xgmi import XgmiCommunicator
    from dtg.utils import comm as dcomm

    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    _, tp_group, _, tp_rank, _ = make_mesh(world)
    cfg = resolve_config("llama-3-8b", num_hidden_layers=layers)
    torch.manual_seed(0)
    model = build_model(cfg, device=dev, tp_group=tp_group)
    dcomm.register_xgmi(tp_group, XgmiCommunicator(tp_group, capacity_bytes=512 << 20, device=dev, gather_engine=engine))
    eng = DataParallel(model, mode="single", tp_group=tp_group, broadcast_from_rank0=False)
    opt = FlatAdamW(eng, lr=1e-5)
    g = torch.Generator().manual_seed(0)
    ids = torch.randint(0, cfg.vocab_size, (batch, seq), generator=g).to(dev)
    res = {}
    for k in chunks_list:
        model.tp.overlap_chunks = k
        for i in range(3 + steps):
            if i == 3:
                torch.cuda.synchronize()
                dist.barrier()
                t0 = time.perf_counter()
            opt.zero_grad()
            out = model(input_ids=ids, labels=ids)
            eng.backward(out.loss)
            opt.step()
        torch.cuda.synchronize()
        dist.barrier()
        res[k] = {"ms_per_step": (time.perf_counter() - t0) * 1e3 / steps, "loss": out.loss.item()}
    dcomm._XGMI[tp_group].check()
    if rank == 0:
        with open(os.path.join(outdir, "result.json"), "w") as f:
            json.dump(res, f)
    dist.barrier()
    dist.destroy_process_group()


def _intervals_overlap(a, bs):
    """Length of interval a covered by the union of sorted, merged intervals bs."""
    s, e = a
    tot = 0
    for bs_, be in bs:
        if be <= s:
            continue
        if bs_ >= e:
            break
        tot += min(e, be) - max(s, bs_)
    return tot


def _merge(iv):
    iv.sort()
    out = []
    for s, e in iv:
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def trace_overlap(d):
    # one CSV per process (rocprofv3 -o %pid%_run): the two ranks share the GPU, so overlap is
    # only meaningful between kernels of the same rank
    by_pid = {}
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        by_pid[os.path.basename(f).split("_")[0]] = list(csv.DictReader(open(f)))
    report = {}
    for pid, rs in by_pid.items():
        comm_iv, comp_iv = [], []
        for r in rs:
            iv = [int(r["Start_Timestamp"]), int(r["End_Timestamp"])]
            name = r["Kernel_Name"]
            if "xgmi" in name:
                if "barrier_kernel" not in name:  # a barrier's spin is waiting, not moving data
                    comm_iv.append(iv)
            elif "copyBuffer" not in name and "fillBuffer" not in name:
                comp_iv.append(iv)
        if not comm_iv:
            continue
        comp = _merge(comp_iv)
        total = sum(e - s for s, e in comm_iv)
        cov = sum(_intervals_overlap((s, e), comp) for s, e in comm_iv)
        report[pid] = {"comm_kernels": len(comm_iv), "comm_ms": total / 1e6,
                       "overlapped_with_compute_ms": cov / 1e6, "overlap_frac": round(cov / max(total, 1), 3)}
    return report


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chunks", type=int, nargs="+", default=[1, 4])
    ap.add_argument("--layers", type=int, default=2)
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--seq", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--out", default="gpurun_out/tp_overlap")
    ap.add_argument("--trace", default=None, help="summarise a rocprofv3 --kernel-trace directory instead")
    ap.add_argument("--engine", default="kernel", choices=["kernel", "dma"], help="xGMI all-gather engine")
    a = ap.parse_args()
    if a.trace:
        print(json.dumps(trace_overlap(a.trace), indent=1))
        return
    import socket

    import torch.multiprocessing as mp

    os.makedirs(a.out, exist_ok=True)
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.start_processes(_worker, args=(2, port, a.chunks, a.layers, a.batch, a.seq, a.steps, a.out, a.engine), nprocs=2,
                       join=True, start_method="spawn")
    print(open(os.path.join(a.out, "result.json")).read())


if __name__ == "__main__":
    main()
