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
(`timeout_s`), the error is sticky (later barriers return at once) and `check()` raises instead
of the GPU hanging.  The trainer calls `utils.comm.check_xgmi()` at every log step, checkpoint
and exit, so a lost peer ends the job with a non-zero exit instead of training on stale data.

Engines: "kernel" pulls with CU kernels over all links at once; "dma" moves every byte with
hipMemcpyAsync on one stream per peer (the copy engines, concurrently, no CU time) and sums the
reduce-scatter's pulled slices with one local kernel.

Zero-copy: `rs_input_buffer()` hands out one of two workspace slots at the END of the
workspace; a producer GEMM writes its output there (`torch.mm(..., out=slot)`) and the
reduce-scatter then skips its stage copy.  A slot is reused only after the reduce-scatter that
read it has passed its closing barrier on this rank (the event recorded by `release_slot`),
which means every peer has finished pulling from it.  Stage copies of other messages start at
offset 0, below the slots.

Fault injection for tests: DTG_XGMI_FAULT="<rank>:<n>" makes group rank <rank> silently skip
its n-th collective (0-based), so its peers' barriers time out (DTG_XGMI_TIMEOUT seconds).
"""
from __future__ import annotations

import os
import socket

import torch
import torch.distributed as dist

from ..ops import _native


class XgmiError(RuntimeError):
    pass


class XgmiCommunicator:
    def __init__(self, group=None, capacity_bytes: int = 64 << 20, device=None, timeout_s: float = None,
                 gather_engine: str = "kernel"):
        """gather_engine: "kernel" (pull kernels over all links at once) or "dma" (hipMemcpyAsync
        copies on per-peer streams, i.e. the copy engines: no CU time, for collectives overlapped
        with GEMMs).  The engine applies to all-gathers and reduce-scatters."""
        _native.require()
        assert gather_engine in ("kernel", "dma"), gather_engine
        self.gather_engine = gather_engine
        if timeout_s is None:
            timeout_s = float(os.environ.get("DTG_XGMI_TIMEOUT", "60"))
        self.timeout_s = float(timeout_s)
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
        self.ws = x.workspace(self.id)  # uint8 view of the own data region
        self._ws_ptr = self.ws.data_ptr()
        self._slot_free = [None, None]  # event after the last reduce-scatter that read each slot
        self._slot_next = 0
        self._slot_of = {}  # data_ptr of a handed-out slot view -> slot index
        self.calls = 0
        self._fault = None
        f = os.environ.get("DTG_XGMI_FAULT")
        if f:
            r, n = (int(v) for v in f.split(":"))
            if r == self.rank:
                self._fault = n
        dist.barrier(group=group)

    # ------------------------------------------------------------------ collectives
    def fits(self, nbytes: int) -> bool:
        return nbytes <= self.capacity and nbytes % 16 == 0

    def _offset(self, t: torch.Tensor) -> int:
        """Byte offset of `t` in the own workspace (zero-copy input), else 0 (staged there)."""
        p = t.data_ptr()
        if self._ws_ptr <= p < self._ws_ptr + self.capacity:
            return p - self._ws_ptr
        return 0

    def _skip(self) -> bool:
        n, self.calls = self.calls, self.calls + 1
        return self._fault is not None and n == self._fault

    def all_gather_into(self, out: torch.Tensor, inp: torch.Tensor) -> torch.Tensor:
        if self._skip():
            return out
        inp = inp.contiguous()
        op = torch.ops.dtg_xgmi.all_gather_dma if self.gather_engine == "dma" else torch.ops.dtg_xgmi.all_gather
        op(self.id, out, inp, self._offset(inp))
        return out

    def reduce_scatter_into(self, out: torch.Tensor, inp: torch.Tensor) -> torch.Tensor:
        if self._skip():
            return out
        inp = inp.contiguous()
        op = torch.ops.dtg_xgmi.reduce_scatter_dma if self.gather_engine == "dma" else torch.ops.dtg_xgmi.reduce_scatter
        op(self.id, out, inp, self._offset(inp))
        return out

    def all_reduce_(self, t: torch.Tensor) -> torch.Tensor:
        assert t.is_contiguous()
        if self._skip():
            return t
        torch.ops.dtg_xgmi.all_reduce(self.id, t, self._offset(t))
        return t

    # ------------------------------------------------------------------ shared buffers
    def alloc_shared(self, nbytes: int) -> tuple:
        """(uint8 tensor, slot): a buffer of `nbytes` that every rank of the group allocates in
        the same call, IPC-exported and mapped from every peer (collective)."""
        x = torch.ops.dtg_xgmi
        t = x.alloc_shared(self.id, int(nbytes))
        slot = getattr(self, "_nshared", 0)
        self._nshared = slot + 1
        mine = bytes(x.shared_handle(self.id, slot).tolist())
        handles = [None] * self.world
        dist.all_gather_object(handles, mine, group=self.group)
        x.open_shared(self.id, slot, torch.tensor([list(h) for h in handles], dtype=torch.uint8))
        return t, slot

    def signal_wait(self):
        """Stream-ordered barrier: returns (on the device) once every peer's stream reached it."""
        if self._skip():
            return
        torch.ops.dtg_xgmi.signal_wait(self.id)

    def pull(self, slot: int, dst: torch.Tensor, src_off, nbytes, dst_off):
        """Copy-engine pulls from every peer's copy of shared `slot` into `dst` (byte ranges)."""
        lt = lambda v: torch.tensor(v, dtype=torch.long)  # noqa: E731
        torch.ops.dtg_xgmi.pull(self.id, slot, dst, lt(src_off), lt(nbytes), lt(dst_off))

    def reduce_pulled(self, out: torch.Tensor, scratch: torch.Tensor, own: torch.Tensor):
        torch.ops.dtg_xgmi.reduce_pulled(self.id, out, scratch, own)

    # ------------------------------------------------------------------ zero-copy slots
    def rs_input_buffer(self, shape, dtype, stage_bytes: int = 0):
        """A workspace view of `shape` for a producer to write a reduce-scatter input into, or
        None if two such slots plus `stage_bytes` of staged messages do not fit.  The current
        stream is made to wait until the slot's previous reduce-scatter has closed."""
        elem = torch.empty((), dtype=dtype).element_size()
        n = 1
        for s_ in shape:
            n *= int(s_)
        nbytes = n * elem
        slot = (nbytes + 4095) // 4096 * 4096
        if 2 * slot + stage_bytes > self.capacity or nbytes % 16:
            return None
        k = self._slot_next
        self._slot_next ^= 1
        ev = self._slot_free[k]
        if ev is not None:
            torch.cuda.current_stream(self.device).wait_event(ev)
            self._slot_free[k] = None
        off = self.capacity - (2 - k) * slot
        self._slot_of[self._ws_ptr + off] = k
        # a distinct base per hand-out (not a view of self.ws): see workspace_view in xgmi.hip
        return torch.ops.dtg_xgmi.workspace_view(self.id, off, [int(x) for x in shape], dtype)

    def release_slot(self, t: torch.Tensor, event):
        """`event` completes once the reduce-scatter reading slot-resident `t` has closed."""
        k = self._slot_of.pop(t.data_ptr(), None)
        if k is not None:
            self._slot_free[k] = event

    def error(self) -> int:
        """0, or 1 + the group rank of the peer a barrier timed out waiting for."""
        if getattr(self, "id", None) is None:
            return 0
        return int(torch.ops.dtg_xgmi.error(self.id))

    def check(self, sync: bool = True):
        """Raise XgmiError if a barrier timed out.  With `sync`, the device is synchronised
        first so every queued collective has run."""
        if getattr(self, "id", None) is None:
            return
        if sync:
            torch.cuda.synchronize(self.device)
        e = self.error()
        if e:
            raise XgmiError(f"xgmi barrier timed out after {self.timeout_s:g} s waiting for peer {e - 1} "
                            f"(group rank {self.rank}); a peer died or fell out of step")

    def close(self):
        if getattr(self, "id", None) is not None:
            torch.cuda.synchronize(self.device)
            torch.ops.dtg_xgmi.destroy(self.id)
            self.id = None
