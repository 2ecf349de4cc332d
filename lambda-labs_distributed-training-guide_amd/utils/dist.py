"""Distributed runtime bootstrap.

One process per GPU.  `init_distributed()` reads the launcher's environment:
  * torchrun / torch.distributed.run (RANK, LOCAL_RANK, WORLD_SIZE, MASTER_ADDR/PORT);
  * SLURM (`SLURM_PROCID`, `SLURM_LOCALID`, `SLURM_NTASKS`) when launched with srun directly;
  * OpenMPI (`OMPI_COMM_WORLD_RANK/SIZE/LOCAL_RANK`) for the mpirun launcher;
  * the deepspeed launcher (`--local_rank` argument, LOCAL_RANK env).
and initialises the process group with the RCCL backend ("nccl" on ROCm) when GPUs are
present, gloo otherwise.  RCCL is initialised eagerly (`device_id=`) so communicator setup is
not charged to the first training step.
"""
from __future__ import annotations

import contextlib
import datetime
import logging
import os
from pathlib import Path
from typing import Optional

import torch
import torch.distributed as dist

LOGGER = logging.getLogger("dtg")


def _env_int(*names, default=None):
    for n in names:
        v = os.environ.get(n)
        if v is not None and v != "":
            return int(v)
    return default


def init_distributed(backend: Optional[str] = None, timeout_minutes: int = 30, local_rank_arg: Optional[int] = None):
    """Initialise torch.distributed from launcher env. Returns (rank, local_rank, world_size, device)."""
    rank = _env_int("RANK", "OMPI_COMM_WORLD_RANK", "SLURM_PROCID", "PMI_RANK", default=0)
    world = _env_int("WORLD_SIZE", "OMPI_COMM_WORLD_SIZE", "SLURM_NTASKS", "PMI_SIZE", default=1)
    # DTG_FAKE_WORLD=W (one process, no launcher): run as rank 0 of a W-rank job whose other ranks
    # are PyTorch's `fake` process group -- every collective returns at once (gathers replicate
    # the local input; utils/comm.py fills the reduce-scatter / all-to-all outputs it leaves
    # untouched).  Shard sizes, gathered buffers, allocations and per-rank compute are those of a
    # real W-rank job; the numerics are not (a memory / per-rank-compute rehearsal only).
    fake_world = int(os.environ.get("DTG_FAKE_WORLD", "0") or 0)
    if fake_world > 1:
        check_fake_world_env(fake_world)
        rank, world = 0, fake_world
    local_rank = local_rank_arg if local_rank_arg is not None else _env_int(
        "LOCAL_RANK", "OMPI_COMM_WORLD_LOCAL_RANK", "SLURM_LOCALID", "MPI_LOCALRANKID", default=None)
    cuda = torch.cuda.is_available()
    ndev = torch.cuda.device_count() if cuda else 1
    if local_rank is None:
        local_rank = rank % max(1, ndev)  # assumes homogeneous nodes (reference B2)
    os.environ.setdefault("RANK", str(rank))
    os.environ.setdefault("WORLD_SIZE", str(world))
    os.environ.setdefault("LOCAL_RANK", str(local_rank))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29500")
    # DTG_SHARED_DEVICE=1: every rank on cuda:0 with gloo collectives -- rehearse a multi-rank
    # layout (real kernels and per-rank shapes, host-staged communication) on a one-GPU machine
    shared = cuda and os.environ.get("DTG_SHARED_DEVICE") == "1"
    device = torch.device("cuda:0" if shared else f"cuda:{local_rank}") if cuda else torch.device("cpu")
    if cuda:
        torch.cuda.set_device(device)
    if fake_world > 1 and not dist.is_initialized():
        from torch.testing._internal.distributed.fake_pg import FakeStore

        os.environ["RANK"], os.environ["WORLD_SIZE"], os.environ["LOCAL_RANK"] = "0", str(world), "0"
        # one node = 8 GPUs (chapter 06's TP degree, HYBRID's shard group)
        os.environ["LOCAL_WORLD_SIZE"] = str(min(world, int(os.environ.get("DTG_FAKE_NODE_GPUS", "8"))))
        dist.init_process_group("fake", store=FakeStore(), rank=0, world_size=world)
        return 0, 0, world, torch.device("cuda:0") if cuda else torch.device("cpu")
    if world > 1 and not dist.is_initialized():
        backend = backend or ("nccl" if cuda and not shared else "gloo")
        timeout = datetime.timedelta(minutes=timeout_minutes)
        kw = dict(backend=backend, rank=rank, world_size=world, timeout=timeout)
        if backend == "nccl":
            kw["device_id"] = device
        store = elastic_store(world, timeout)
        if store is not None:
            kw["store"] = store
        dist.init_process_group(**kw)
    return rank, local_rank, world, device


def elastic_store(world: int, timeout):
    """Under torchrun: the agent's TCPStore with a per-restart-attempt key prefix, else None.

    torchrun keeps one agent-hosted store for every restart of the worker group and the env://
    rendezvous adds no per-attempt prefix, so after an elastic restart the
    process-group bootstrap can read a previous attempt's keys -- gloo's full-mesh connect then
    dials a dead worker's port and every later attempt inherits the stale keys
    (tests/test_elastic_cpu.py reproduced it under load).  Attempt N's keys live under
    attempt_N here."""
    if os.environ.get("TORCHELASTIC_USE_AGENT_STORE") != "True" or "MASTER_ADDR" not in os.environ:
        return None
    store = dist.TCPStore(os.environ["MASTER_ADDR"], int(os.environ["MASTER_PORT"]), world, is_master=False,
                          timeout=timeout)
    return dist.PrefixStore(f"dtg/attempt_{os.environ.get('TORCHELASTIC_RESTART_COUNT', '0')}", store)


def fake_world() -> int:
    """W of a DTG_FAKE_WORLD=W one-rank rehearsal, else 0."""
    return int(os.environ.get("DTG_FAKE_WORLD", "0") or 0)


def check_fake_world_env(fake: int, env=None) -> None:
    """A rehearsal is ONE process.  DTG_FAKE_WORLD leaking into a real launcher's job would turn
    every rank into "rank 0 on cuda:0" training on no-op collectives without an error, so it is
    refused whenever a launcher says this process is one of several."""
    env = os.environ if env is None else env
    if "TORCHELASTIC_RUN_ID" in env:
        raise RuntimeError("DTG_FAKE_WORLD is set inside a torchrun job; unset it (rehearsals are one process)")
    for k in ("WORLD_SIZE", "OMPI_COMM_WORLD_SIZE", "SLURM_NTASKS", "PMI_SIZE"):
        v = env.get(k)
        if v not in (None, "") and int(v) > 1 and int(v) != fake:
            raise RuntimeError(f"DTG_FAKE_WORLD={fake} but the launcher set {k}={v}; unset DTG_FAKE_WORLD")


def get_rank() -> int:
    return dist.get_rank() if dist.is_initialized() else 0


def get_world_size() -> int:
    return dist.get_world_size() if dist.is_initialized() else 1


def barrier(group=None):
    if dist.is_initialized():
        dist.barrier(group=group)


@contextlib.contextmanager
def rank_ordered(should_go_first: bool, group=None):
    """Ranks with should_go_first run the body, then a barrier releases the others (B5)."""
    if should_go_first:
        yield
    barrier(group)
    if not should_go_first:
        yield
    barrier(group)


@contextlib.contextmanager
def rank0_first(group=None):
    """Rank 0 runs the body first (downloads, cache writes), then everyone else (B4)."""
    with rank_ordered(get_rank() == 0, group):
        yield


def local_rank0_first():
    return rank_ordered(int(os.environ.get("LOCAL_RANK", "0")) == 0)


def is_shared_fs(path) -> bool:
    """True if `path` lives on a network/shared mount (walks up to the mount point).

    The reference tests `exp_dir.is_mount()` on the leaf directory, which is almost always False
    (SURVEY §2.11 #10); this finds the filesystem that actually contains the path."""
    p = Path(path).resolve()
    while not p.exists():
        p = p.parent
    while not os.path.ismount(p):
        p = p.parent
    try:
        with open("/proc/mounts") as fp:
            for line in fp:
                parts = line.split()
                if len(parts) >= 3 and parts[1] == str(p):
                    return parts[2] in ("nfs", "nfs4", "lustre", "beegfs", "gpfs", "cifs", "fuse.sshfs", "ceph", "wekafs")
    except OSError:
        pass
    return False


def make_exp_dir(exp_dir, per_rank_dirs: bool = False):
    """Create the experiment directory race-free: one writer per filesystem, barriers around (B6)."""
    exp_dir = Path(exp_dir)
    barrier()
    writer = get_rank() == 0 if is_shared_fs(exp_dir.parent if not exp_dir.exists() else exp_dir) \
        else int(os.environ.get("LOCAL_RANK", "0")) == 0
    if writer:
        exp_dir.mkdir(parents=True, exist_ok=True)
    barrier()
    if per_rank_dirs:
        (exp_dir / f"rank-{get_rank()}").mkdir(parents=True, exist_ok=True)
    barrier()
    return exp_dir


def _parse_cpulist(text: str):
    cpus = set()
    for part in text.strip().split(","):
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-")
            cpus.update(range(int(a), int(b) + 1))
        else:
            cpus.add(int(part))
    return cpus


def host_placement(device, pin: bool = False, share: int = 0) -> dict:
    """Where this rank's host work runs relative to its GPU: the CPUs it may use
    (`os.sched_getaffinity`), the GPU's NUMA node and that node's CPUs (sysfs, from the PCI bus
    id), and OMP_NUM_THREADS.  Chapter 05's backward is bound by gradient D2H and the host AdamW
    runs on these CPUs, so the numbers are logged at startup; `pin=True` restricts the process
    to the GPU-local NUMA node's CPUs (within its current affinity) so pinned buffers, the DMA
    engine and the optimizer threads share one memory controller."""
    info = {"affinity_cpus": None, "gpu_numa_node": None, "numa_cpus": None, "omp_threads": os.environ.get("OMP_NUM_THREADS")}
    try:
        aff = os.sched_getaffinity(0)
        info["affinity_cpus"] = len(aff)
    except (AttributeError, OSError):
        aff = None
    if getattr(device, "type", "cpu") == "cuda":
        try:
            bus = torch.cuda.get_device_properties(device).pci_bus_id  # bus number, e.g. 93 = 0000:5d:..

            def _is_gpu(d):  # display / processing-accelerator class on that bus
                c = d / "class"
                return c.exists() and c.read_text().strip()[:4] in ("0x03", "0x12")

            dev_dirs = [d for d in Path("/sys/bus/pci/devices").iterdir()
                        if int(d.name.split(":")[1], 16) == int(bus) and _is_gpu(d)]
            for d in dev_dirs:
                node_file = d / "numa_node"
                if node_file.exists():
                    node = int(node_file.read_text().strip())
                    if node >= 0:
                        info["gpu_numa_node"] = node
                        cl = Path(f"/sys/devices/system/node/node{node}/cpulist")
                        if cl.exists():
                            cpus = _parse_cpulist(cl.read_text())
                            info["numa_cpus"] = len(cpus)
                            if aff is not None:
                                info["affinity_cpus_on_gpu_node"] = len(cpus & aff)
                                if pin and cpus & aff:
                                    os.sched_setaffinity(0, cpus & aff)
                                    info["pinned_to_gpu_node"] = True
                                    info["affinity_cpus"] = len(cpus & aff)
                    break
        except Exception as e:  # informational only: never fail a run over sysfs layout
            info["error"] = repr(e)[:120]
    if share and share > 0:
        # one rank's share of a node's cores (threads created from here on inherit it)
        try:
            cur = sorted(os.sched_getaffinity(0))
            keep = set(cur[:share])
            os.sched_setaffinity(0, keep)
            torch.set_num_threads(len(keep))
            info["cpu_share"] = len(keep)
            info["affinity_cpus"] = len(keep)
        except (AttributeError, OSError) as e:
            info["cpu_share_error"] = repr(e)[:120]
    return info


def setup_logging(rank: Optional[int] = None, with_rank: bool = True):
    """Reference log format: `[rank=R] [time] LEVEL:message` (B8)."""
    rank = get_rank() if rank is None else rank
    fmt = f"[rank={rank}] [%(asctime)s] %(levelname)s:%(message)s" if with_rank else "[%(asctime)s] %(levelname)s:%(message)s"
    logging.basicConfig(format=fmt, level=logging.INFO, force=True)
    return LOGGER


def record(fn):
    """@record from torch.distributed.elastic: writes the failing worker's traceback to
    $TORCHELASTIC_ERROR_FILE (B7)."""
    try:
        from torch.distributed.elastic.multiprocessing.errors import record as _record

        return _record(fn)
    except Exception:  # pragma: no cover
        return fn


def device_mesh_2d(tp: int, device_type: Optional[str] = None):
    """(dp, tp) groups for tensor/2-D parallelism; tp ranks are contiguous (one xGMI island)."""
    world = get_world_size()
    assert world % tp == 0, f"world size {world} not divisible by tp={tp}"
    from torch.distributed.device_mesh import init_device_mesh

    device_type = device_type or ("cuda" if torch.cuda.is_available() else "cpu")
    mesh = init_device_mesh(device_type, (world // tp, tp), mesh_dim_names=("dp", "tp"))
    return mesh
