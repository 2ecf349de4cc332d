"""Tensor/sequence-parallel regions with their collectives overlapped by compute (async TP).

A Megatron sequence-parallel sub-block is

    x_local [T/n, H] --all-gather--> x [T, H] --f--> y partial [T, H] --reduce-scatter--> [T/n, H]

where f is the column-parallel -> row-parallel pair (QKV -> attention -> o_proj, or
gate_up -> SwiGLU -> down).  Run as written (`tp_comm.gather_seq` / `scatter_seq`), the
all-gather and the reduce-scatter sit on the critical path, with every GEMM waiting for the
whole gather and the scatter waiting for the last GEMM.

`sp_region` cuts this rank's T/n rows into k chunks and pipelines them:

    forward   AG(0) | AG(1) f(0) | RS(0) AG(2) f(1) | RS(1) AG(3) f(2) | ... | RS(k-1)
    backward  the same shape: AG(dY chunk) -> f's backward -> RS(dX chunk)

Chunk j of the gathered tensor is the j-th chunk of every rank ([n * T/(n k), H], rank-major),
and f is row-local, so y's chunk j reduce-scatters straight into this rank's j-th output chunk:
no reordering copies.  Collectives are issued with async_op on RCCL (its own stream) or on a
side stream for the direct-peer xGMI library (utils/comm.py), and waited for only right
before the GEMM that consumes them.  Only the first gather and the last scatter of a region
stay exposed (2/k of the traffic instead of all of it).

With the direct-peer xGMI library registered for the group, the forward's row-parallel GEMM of
chunk j writes its partial output straight into one of two workspace slots
(`XgmiCommunicator.rs_input_buffer`), so the reduce-scatter pulls from it without a stage copy.
fn(x, j, out=None) must honour `out` for that (LlamaAttention / LlamaMLP do).

Each chunk's f is recorded as its own small autograd graph inside the region's forward;
the region's backward replays them chunk by chunk between the collectives.  Weight gradients
from the k chunks accumulate in `main_grad` (first chunk writes, later chunks add), and the
engines' "gradient final" notifications are deferred to the end of the region, so DDP / ZeRO /
FSDP buckets fire once per weight as before.

Attention chunks must hold whole sequences (dense rows, T/n a multiple of k x S); the MLP
region accepts any chunking.  Layers under activation checkpointing keep the synchronous
path (a recompute must not stop half-way through a pipelined region).

With `regather` (`--sp-regather on`), autograd does not keep the GATHERED chunk for the
column-parallel GEMM's weight gradient: a saved-tensor hook swaps it for a handle on this rank's
local rows, and the backward re-gathers them (prefetched with the chunk's dY gather).  The
activations a layer keeps shrink by (1 - 1/n) of one [T, H] tensor per region -- at the 405B
tp 4 recipe 0.4 GB per region -- for one more all-gather per region in the backward, which is
what lets `--ac-layers auto` release more layers from recomputation (`regathered`).

Reference behaviour: the reference's TP chapter runs DTensor's synchronous redistributes
(/root/reference/06-tensor-parallel/train_llm.py:84-128); this is the MI355X design that hides
them, not a translation.
"""
from __future__ import annotations

import contextlib
import os

import torch

from ..ops.grad_routing import deferred_notifications
from ..utils import comm

DEFAULT_CHUNKS = int(os.environ.get("DTG_TP_OVERLAP_CHUNKS", "2"))


class RegatherHandle:
    """A sequence-parallel all-gather result [n * c, ...] that autograd does not keep: `get()`
    re-gathers this rank's `local` rows (waiting for a `prefetch()` issued earlier, if any)."""

    def __init__(self, local, shape, dtype, group):
        self.local, self.shape, self.dtype, self.group = local, tuple(shape), dtype, group
        self._buf = self._work = None

    def prefetch(self):
        if self._buf is None:
            self._buf = torch.empty(self.shape, dtype=self.dtype, device=self.local.device)
            self._work = comm.all_gather_dim0_into_async(self._buf, self.local, self.group)

    def get(self):
        """The re-gathered tensor.  The handle drops its own reference: the tensor lives only as
        long as the backward node that unpacked it (autograd keeps the graph's nodes -- and the
        handles they reference -- until the step's output is released)."""
        self.prefetch()
        if self._work is not None:
            self._work.wait()
            self._work = None
        buf, self._buf = self._buf, None
        return buf


@contextlib.contextmanager
def regathered(full, local, group):
    """Inside the block, every tensor autograd saves that IS `full` (same storage, shape, strides and
    dtype: the gathered activation the column-parallel GEMM keeps for its weight gradient) is
    replaced by a RegatherHandle on `local`; the backward's unpack re-gathers it.  Yields the
    handle (callers prefetch it ahead of the backward that needs it)."""
    h = RegatherHandle(local, full.shape, full.dtype, group)
    key = (full.data_ptr(), tuple(full.shape), tuple(full.stride()), full.dtype)

    def pack(t):
        if (t.data_ptr(), tuple(t.shape), tuple(t.stride()), t.dtype) == key:
            return h
        return t

    def unpack(v):
        return v.get() if isinstance(v, RegatherHandle) else v

    with torch.autograd.graph.saved_tensors_hooks(pack, unpack):
        yield h


class _Region(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, fn, group, k, regather, *params):
        n = comm.world(group)
        Tl, H = x.shape
        Tc = Tl // k
        xs = x.contiguous().view(k, Tc, H)
        out = torch.empty_like(xs)
        g = torch.empty((n * Tc, H), dtype=x.dtype, device=x.device)
        work = comm.all_gather_dim0_into_async(g, xs[0], group)
        leaves, ys, rs, handles, in_slot = [], [], [], [], []
        for j in range(k):
            work.wait()
            cur = g
            if j + 1 < k:  # prefetch the next chunk while this one computes
                g = torch.empty((n * Tc, H), dtype=x.dtype, device=x.device)
                work = comm.all_gather_dim0_into_async(g, xs[j + 1], group)
            # zero-copy: the chunk's row-parallel GEMM writes straight into an xGMI workspace slot
            buf = comm.rs_input_buffer(group, (n * Tc, H), x.dtype, stage_bytes=Tc * H * x.element_size())
            with torch.enable_grad():
                leaf = cur.detach().requires_grad_(True)
                with (regathered(leaf, xs[j], group) if regather else contextlib.nullcontext()) as h:
                    y = fn(leaf, j) if buf is None else fn(leaf, j, out=buf)
            rs.append(comm.reduce_scatter_dim0_into_async(out[j], y.detach(), group))
            leaves.append(leaf)
            ys.append(y)
            handles.append(h)
            in_slot.append(buf is not None)
        for w in rs:
            w.wait()
        # The chunks' partial outputs have been reduce-scattered: their backward needs only their
        # graphs, not their values, so the [n * Tc, H] buffers go now instead of at the backward
        # (xGMI workspace slots are the communicator's and stay).
        for y, slot in zip(ys, in_slot):
            if not slot:
                y.untyped_storage().resize_(0)
        if regather:  # the gathered chunks are dropped: the leaves keep only their metadata (for .grad)
            for leaf in leaves:
                leaf.untyped_storage().resize_(0)
            ctx.xs = xs
        ctx.leaves, ctx.ys, ctx.group, ctx.k, ctx.n_params = leaves, ys, group, k, len(params)
        ctx.handles = handles
        return out.view(Tl, H)

    @staticmethod
    def backward(ctx, dout):
        group, k = ctx.group, ctx.k
        n = comm.world(group)
        Tl, H = dout.shape
        Tc = Tl // k
        ds = dout.contiguous().view(k, Tc, H)
        dx = torch.empty_like(ds)
        g = torch.empty((n * Tc, H), dtype=dout.dtype, device=dout.device)
        work = comm.all_gather_dim0_into_async(g, ds[0], group)
        hs = ctx.handles
        if hs[0] is not None:
            hs[0].prefetch()
        rs = []
        with deferred_notifications():
            for j in range(k):
                work.wait()
                cur = g
                if j + 1 < k:
                    g = torch.empty((n * Tc, H), dtype=dout.dtype, device=dout.device)
                    work = comm.all_gather_dim0_into_async(g, ds[j + 1], group)
                    if hs[j + 1] is not None:
                        hs[j + 1].prefetch()
                y, leaf = ctx.ys[j], ctx.leaves[j]
                torch.autograd.backward(y, cur)
                gx = leaf.grad
                ctx.ys[j] = ctx.leaves[j] = hs[j] = None  # release chunk j's graph and saved activations
                rs.append(comm.reduce_scatter_dim0_into_async(dx[j], gx, group))
                del y, leaf, gx
            for w in rs:
                w.wait()
        ctx.xs = ctx.handles = None
        return (dx.view(Tl, H), None, None, None, None) + (None,) * ctx.n_params


def sp_region(x, fn, group, k, params, regather: bool = False):
    """reduce_scatter(fn(all_gather(x))) with k-chunk compute/communication overlap.

    fn(x_chunk_gathered, j[, out=buffer]) -> partial output of the same row count (written into
    `out` when one is passed); `params` are the weights
    fn uses (passed so the region is part of the autograd graph even when x needs no grad).
    regather: re-gather the chunks in the backward instead of keeping them (see the module doc)."""
    return _Region.apply(x, fn, group, int(k), bool(regather), *params)


def region_chunks(rows_local: int, k: int, row_len: int = 1) -> int:
    """Largest chunk count <= k that splits rows_local into whole `row_len` multiples (1 = off)."""
    units = rows_local // row_len if row_len and rows_local % row_len == 0 else 0
    for c in range(max(1, k), 1, -1):
        if units and units % c == 0:
            return c
    return 1
