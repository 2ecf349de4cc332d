"""ZeRO's bucket collectives on the xGMI copy engines (`--dp-comm xgmi-dma`).

RCCL's reduce-scatter / all-gather kernels run on CUs, so every gradient bucket reduced during
the backward and every parameter bucket gathered under the next forward takes compute units
from the GEMMs it is meant to hide under.  On one MI355X node the 8 GPUs are fully connected by
point-to-point xGMI links and every GPU has copy engines that move data over them without
touching the shader array.  This module runs ZeRO's traffic there, zero-copy:

* the engine's flat parameter and gradient buffers are allocated through the xGMI library
  (`XgmiCommunicator.alloc_shared`) and every rank maps every peer's copy;
* gradient reduce-scatter of bucket b: after a stream-ordered barrier (every rank's backward has
  written b), this rank pulls ITS slice of b from each of the 7 peers' gradient buffers -- one
  hipMemcpyAsync per peer, each on its own stream, i.e. one copy engine and one xGMI link per
  peer, all at once -- into a scratch, and one local kernel sums the 8 slices (f32 accumulation,
  rank order) into the gradient shard;
* parameter all-gather of bucket b: after a barrier (every rank's AdamW has updated its slice),
  this rank pulls every peer's updated slice straight into place in its own parameter buffer:
  no staging, no copy-out.

Only the one-wave barrier kernel and the local sum touch CUs.  Each direction has its own
communicator (own signal rows and epochs) and its own side stream; work objects expose the same
`wait()` the RCCL ones do (the caller's stream waits on an event, the host never blocks).

No "done" barrier is needed after the pulls: a peer next writes the gradient bucket a rank
pulled from only in its next backward, which follows its forward, which waited for its
all-gather of that bucket, whose barrier requires every rank to have finished its AdamW of the
bucket -- which follows that rank's reduce-scatter pulls on its stream.  Symmetrically a peer's
next AdamW of a parameter slice follows the next reduce-scatter barrier of the bucket, which
every rank reaches only after its forward consumed (i.e. waited for) its gather of it.

RCCL stays the default and the inter-node path; all ranks of the group must share a node.
"""
from __future__ import annotations

import torch

from .xgmi import XgmiCommunicator


class _EventWork:
    """RCCL-work-like handle of a side-stream collective: wait() makes the CURRENT stream wait."""

    def __init__(self, ev: torch.cuda.Event, device):
        self.ev = ev
        self.device = device

    def wait(self):
        torch.cuda.current_stream(self.device).wait_event(self.ev)
        return True

    def is_completed(self):
        return self.ev.query()


class XgmiZero:
    def __init__(self, group, device, timeout_s: float = None):
        self.device = torch.device(device)
        # one communicator per direction: separate signal rows / epochs for the two side streams
        self.rs = XgmiCommunicator(group, capacity_bytes=4096, device=self.device, gather_engine="dma",
                                   timeout_s=timeout_s)
        self.ag = XgmiCommunicator(group, capacity_bytes=4096, device=self.device, gather_engine="dma",
                                   timeout_s=timeout_s)
        self.world, self.rank = self.rs.world, self.rs.rank
        from ..utils import comm as _comm

        _comm.register_xgmi_health(self.rs)  # a lost peer ends the trainer at the step (poll_xgmi)
        _comm.register_xgmi_health(self.ag)
        self.rs_stream = torch.cuda.Stream(device=self.device)
        self.ag_stream = torch.cuda.Stream(device=self.device)
        self._slot = {}

    def alloc(self, numel: int, dtype, kind: str) -> torch.Tensor:
        """Flat buffer `kind` ("param" | "grad") in IPC-shared memory (collective)."""
        esz = torch.empty((), dtype=dtype).element_size()
        comm = self.ag if kind == "param" else self.rs
        raw, slot = comm.alloc_shared(max(16, numel * esz))
        self._slot[kind] = slot
        return raw[: numel * esz].view(dtype)

    def reduce_scatter(self, grad_buf: torch.Tensor, ranges, out: torch.Tensor) -> _EventWork:
        """out = sum over ranks of their grad_buf[ranges[self.rank]]; ranges[r] = (start, end) of
        rank r's slice of the bucket (elements of the flat buffer)."""
        s, e = ranges[self.rank]
        n = e - s
        esz = grad_buf.element_size()
        st = self.rs_stream
        st.wait_stream(torch.cuda.current_stream(self.device))  # this bucket's gradients are written
        with torch.cuda.stream(st):
            self.rs.signal_wait()  # ... on every rank
            scratch = torch.empty(self.world * n, dtype=grad_buf.dtype, device=self.device)
            nbytes = [0 if r == self.rank else n * esz for r in range(self.world)]
            self.rs.pull(self._slot["grad"], scratch, [s * esz] * self.world, nbytes,
                         [r * n * esz for r in range(self.world)])
            self.rs.reduce_pulled(out, scratch, grad_buf[s:e])
            ev = torch.cuda.Event()
            ev.record(st)
        return _EventWork(ev, self.device)

    def all_gather(self, param_buf: torch.Tensor, ranges) -> _EventWork:
        """Every peer's updated slice ranges[r] of param_buf pulled into place."""
        esz = param_buf.element_size()
        st = self.ag_stream
        st.wait_stream(torch.cuda.current_stream(self.device))  # this rank's update of its slice
        with torch.cuda.stream(st):
            self.ag.signal_wait()  # ... and every peer's
            offs = [a * esz for a, _ in ranges]
            nbytes = [0 if r == self.rank else (b - a) * esz for r, (a, b) in enumerate(ranges)]
            self.ag.pull(self._slot["param"], param_buf, offs, nbytes, offs)
            ev = torch.cuda.Event()
            ev.record(st)
        return _EventWork(ev, self.device)

    def check(self, sync: bool = True):
        self.rs.check(sync)
        self.ag.check(sync)

    def close(self):
        self.rs.close()
        self.ag.close()


class XgmiFsdp:
    """FSDP (ZeRO-3) unit collectives on the copy engines (`FullyShard(dp_comm="xgmi-dma")`).

    * all-gather of a unit: after a barrier, pull every peer's shard of the unit from its shared
      parameter-shard buffer straight into this rank's gathered unit buffer (own shard: a local
      copy on the same side stream);
    * reduce-scatter of a unit's gradient: the backward writes the unit's full gradient into one of
      `nslots` slots of a shared gradient pool; after a barrier every rank pulls its slice of the
      slot from each peer and sums it locally; a second barrier ("every peer has pulled from this
      slot") releases the slot, and the backward that next writes into it waits for that event.

    A parameter shard needs no release barrier (its owner next updates it only after the unit's
    reduce-scatter barrier, which every rank reaches after its own gathers of the unit)."""

    def __init__(self, group, device, nslots: int = 4, timeout_s: float = None):
        self.device = torch.device(device)
        self.ag = XgmiCommunicator(group, capacity_bytes=4096, device=self.device, gather_engine="dma",
                                   timeout_s=timeout_s)
        self.rs = XgmiCommunicator(group, capacity_bytes=4096, device=self.device, gather_engine="dma",
                                   timeout_s=timeout_s)
        from ..utils import comm as _comm

        _comm.register_xgmi_health(self.ag)
        _comm.register_xgmi_health(self.rs)
        self.world, self.rank = self.ag.world, self.ag.rank
        self.ag_stream = torch.cuda.Stream(device=self.device)
        self.rs_stream = torch.cuda.Stream(device=self.device)
        self.nslots = nslots
        self._shard_slot = None
        self._pool = None

    def alloc_shards(self, numel: int, dtype) -> torch.Tensor:
        esz = torch.empty((), dtype=dtype).element_size()
        raw, self._shard_slot = self.ag.alloc_shared(max(16, numel * esz))
        return raw[: numel * esz].view(dtype)

    def alloc_grad_pool(self, slot_numel: int, dtype):
        esz = torch.empty((), dtype=dtype).element_size()
        self.slot_numel = (slot_numel + 7) // 8 * 8
        raw, self._pool_slot = self.rs.alloc_shared(self.nslots * self.slot_numel * esz)
        self._pool = raw[: self.nslots * self.slot_numel * esz].view(dtype)
        self._free = [None] * self.nslots  # event: every peer pulled from the slot
        self._held = [False] * self.nslots  # acquired by a unit whose reduce-scatter is not issued yet
        self._next = 0

    def grad_buffer(self, numel: int):
        """(view of the next free pool slot, slot index); the current stream waits until every
        peer has finished pulling the slot's previous contents.  Slots still held by a unit whose
        reduce-scatter has not been issued (the root unit holds one from its forward to the end of
        the backward) are skipped; the choice depends only on program order, so every rank picks
        the same slot for the same unit."""
        for _ in range(self.nslots):
            k = self._next
            self._next = (k + 1) % self.nslots
            if not self._held[k]:
                break
        else:
            raise RuntimeError(f"XgmiFsdp: all {self.nslots} gradient-pool slots are held by units whose "
                               "reduce-scatter has not been issued")
        self._held[k] = True
        ev = self._free[k]
        if ev is not None:
            torch.cuda.current_stream(self.device).wait_event(ev)
            self._free[k] = None
        o = k * self.slot_numel
        return self._pool[o:o + numel], k

    def gather(self, full: torch.Tensor, shard_off: int, n: int, own: torch.Tensor) -> _EventWork:
        esz = full.element_size()
        st = self.ag_stream
        st.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(st):
            self.ag.signal_wait()
            full[self.rank * n:(self.rank + 1) * n].copy_(own)
            nbytes = [0 if r == self.rank else n * esz for r in range(self.world)]
            self.ag.pull(self._shard_slot, full, [shard_off * esz] * self.world, nbytes,
                         [r * n * esz for r in range(self.world)])
            ev = torch.cuda.Event()
            ev.record(st)
        return _EventWork(ev, self.device)

    def reduce_scatter(self, k: int, n: int, out: torch.Tensor) -> _EventWork:
        self._held[k] = False  # released to the ring; reuse waits for this call's release event
        esz = self._pool.element_size()
        base = k * self.slot_numel
        st = self.rs_stream
        st.wait_stream(torch.cuda.current_stream(self.device))  # the unit's gradient is written
        with torch.cuda.stream(st):
            self.rs.signal_wait()
            scratch = torch.empty(self.world * n, dtype=self._pool.dtype, device=self.device)
            nbytes = [0 if r == self.rank else n * esz for r in range(self.world)]
            self.rs.pull(self._pool_slot, scratch, [(base + self.rank * n) * esz] * self.world, nbytes,
                         [r * n * esz for r in range(self.world)])
            self.rs.reduce_pulled(out, scratch, self._pool[base + self.rank * n:base + (self.rank + 1) * n])
            self.rs.signal_wait()  # every peer has pulled from this slot: it may be rewritten
            ev = torch.cuda.Event()
            ev.record(st)
        self._free[k] = ev
        return _EventWork(ev, self.device)

    def check(self, sync: bool = True):
        self.ag.check(sync)
        self.rs.check(sync)
