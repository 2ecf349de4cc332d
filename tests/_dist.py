"""Helpers to run a function on W CPU ranks (gloo) and collect per-rank results."""
import os
import socket
import tempfile

import torch
import torch.multiprocessing as mp


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _entry(rank, world, port, fn, args, outdir, backend="gloo"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    # c10d's collective-consistency checks (every collective's op / shape / dtype is
    # fingerprinted and compared across ranks) catch mismatched collectives in the engines.
    os.environ.setdefault("TORCH_DISTRIBUTED_DEBUG", "DETAIL")
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    if root not in sys.path:
        sys.path.insert(0, root)
    import dtg  # noqa: F401
    import torch.distributed as dist

    torch.set_num_threads(1)
    if backend == "nccl":  # RCCL: one rank per device (the 1-GPU box runs world 1)
        torch.cuda.set_device(rank)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", rank))
    else:
        dist.init_process_group(backend, rank=rank, world_size=world)
    try:
        res = fn(rank, world, *args)
        torch.save(res, os.path.join(outdir, f"r{rank}.pt"))
    finally:
        dist.destroy_process_group()


def run_distributed(fn, world, *args, backend="gloo"):
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_entry, args=(world, free_port(), fn, args, d, backend), nprocs=world, join=True,
                           start_method="spawn")
        return [torch.load(os.path.join(d, f"r{r}.pt"), weights_only=False) for r in range(world)]
