"""Direct-peer xGMI collectives for tensor/sequence-parallel traffic.

`XgmiCommunicator` wraps the HIP library in csrc/comm/xgmi.hip: one IPC-shared workspace per
rank, every rank maps all peers' workspaces, and all-gather / reduce-scatter / all-reduce pull
from the 7 peers concurrently (one xGMI link each) instead of stepping around a ring.  It is
meant for the TP/SP activation messages (MiBs to tens of MiBs, latency- and link-bound), not
for the large DDP/ZeRO/FSDP gradient buckets, which stay on RCCL.

    comm = XgmiCommunicator(tp_group, capacity_bytes=64 << 20)
    dtg.utils.comm.register_xgmi(tp_group, comm)   # tp_comm's AG/RS/AR now use it

All ranks of the group must sit on one node (xGMI island); the constructor checks that.  The
communicator is stream-ordered on the caller's current stream like an RCCL call with
async_op=False; a peer that never arrives at a barrier trips a bounded wait inside the kernel
(`timeout_s`) and `check()` raises instead of the GPU hanging.
"""
from __future__ import annotations

import socket

import torch
import torch.distributed as dist

from ..ops import _native


class XgmiError(RuntimeError):
    pass


class XgmiCommunicator:
    def __init__(self, group=None, capacity_bytes: int = 64 << 20, device=None, timeout_s: float = 10.0,
                 gather_engine: str = "kernel"):
        """gather_engine: "kernel" (pull kernels over all links at once) or "dma" (hipMemcpyAsync
        copies on the copy engines: no CU time, for all-gathers overlapped with GEMMs)."""
        _native.require()
        assert gather_engine in ("kernel", "dma"), gather_engine
        self.gather_engine = gather_engine
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = torch.device(device)
        hosts = [None] * self.world
        dist.all_gather_object(hosts, socket.gethostname(), group=group)
        if len(set(hosts)) != 1:
            raise XgmiError(f"xgmi communicator spans several hosts {sorted(set(hosts))}; use RCCL across nodes")
        self.capacity = (int(capacity_bytes) + 4095) // 4096 * 4096
        x = torch.ops.dtg_xgmi
        self.id = x.create(self.capacity, self.rank, self.world, self.device.index)
        x.set_timeout(self.id, float(timeout_s))
        mine = bytes(x.ipc_handle(self.id).tolist())
        handles = [None] * self.world
        dist.all_gather_object(handles, mine, group=group)
        table = torch.tensor([list(h) for h in handles], dtype=torch.uint8)
        x.open_peers(self.id, table)
        dist.barrier(group=group)

    # ------------------------------------------------------------------ collectives
    def fits(self, nbytes: int) -> bool:
        return nbytes <= self.capacity and nbytes % 16 == 0

    def all_gather_into(self, out: torch.Tensor, inp: torch.Tensor) -> torch.Tensor:
        op = torch.ops.dtg_xgmi.all_gather_dma if self.gather_engine == "dma" else torch.ops.dtg_xgmi.all_gather
        op(self.id, out, inp.contiguous())
        return out

    def reduce_scatter_into(self, out: torch.Tensor, inp: torch.Tensor) -> torch.Tensor:
        torch.ops.dtg_xgmi.reduce_scatter(self.id, out, inp.contiguous())
        return out

    def all_reduce_(self, t: torch.Tensor) -> torch.Tensor:
        assert t.is_contiguous()
        torch.ops.dtg_xgmi.all_reduce(self.id, t)
        return t

    def check(self):
        """Raise if a barrier timed out (call after a device synchronize)."""
        e = torch.ops.dtg_xgmi.error(self.id)
        if e:
            raise XgmiError(f"xgmi barrier timed out waiting for peer {e - 1} (rank {self.rank})")

    def close(self):
        if getattr(self, "id", None) is not None:
            torch.cuda.synchronize(self.device)
            torch.ops.dtg_xgmi.destroy(self.id)
            self.id = None
