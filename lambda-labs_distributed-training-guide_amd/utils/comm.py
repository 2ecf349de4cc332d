"""Collective primitives over torch.distributed (RCCL on MI355X, gloo on CPU).

Thin helpers that pick the native collective where the backend has it: RCCL implements
`all_gather_into_tensor` / `reduce_scatter_tensor` directly; gloo (CPU tests) lacks
reduce-scatter, so it is expressed as all-reduce + local slice there.  These helpers are used
by the TP/SP functions and the DDP/ZeRO/FSDP engines.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def backend_of(group=None) -> str:
    return dist.get_backend(group)


def world(group=None) -> int:
    return dist.get_world_size(group) if dist.is_initialized() else 1


def rank(group=None) -> int:
    return dist.get_rank(group) if dist.is_initialized() else 0


# Direct-peer xGMI communicators (dtg.parallel.xgmi) registered per process group: the TP/SP
# helpers below route GPU messages that fit the communicator's workspace through them and
# everything else through RCCL.
_XGMI = {}


def register_xgmi(group, communicator):
    _XGMI[group] = communicator


def unregister_xgmi(group):
    return _XGMI.pop(group, None)


# Communicators that carry no TP/SP traffic but must be health-checked too (the data-parallel
# copy-engine path, parallel/xgmi_dp.py).
_XGMI_HEALTH = []


def register_xgmi_health(communicator):
    _XGMI_HEALTH.append(communicator)


def check_xgmi():
    """Raise XgmiError if any registered direct-peer communicator saw a barrier time out (a
    peer died or fell out of step).  Synchronises the device.  Called by the trainer at every
    log step, checkpoint and exit."""
    for c in list(_XGMI.values()) + [c for c in _XGMI_HEALTH if getattr(c, "id", None) is not None]:
        c.check()


def poll_xgmi():
    """Like check_xgmi() but without synchronising the device: reads each communicator's
    host-pinned error word (written by a barrier kernel that timed out).  Cheap enough for
    every training step."""
    for c in list(_XGMI.values()) + [c for c in _XGMI_HEALTH if getattr(c, "id", None) is not None]:
        c.check(sync=False)


def rs_input_buffer(group, shape, dtype, stage_bytes: int = 0):
    """Zero-copy reduce-scatter input: a workspace slot of the group's xGMI communicator for a
    producer to write into, or None (no communicator / does not fit)."""
    c = _XGMI.get(group)
    if c is None or world(group) == 1:
        return None
    return c.rs_input_buffer(shape, dtype, stage_bytes)


# DTG_FAKE_WORLD rehearsals (utils/dist.py): the fake process group returns at once.  Its
# gathers write the local input into every chunk of the output, but its reduce-scatters and
# all-to-alls leave the output untouched: uninitialised memory, whose bf16 reading holds NaN / Inf
# patterns that poison the run (and NaN operands draw less power in the power-limited GEMMs, so
# a rehearsal on them times 12-14 % fast, profiles/r5/405b_fill/).  These fills stand in for the
# other ranks with this rank's data: a reduce-scatter keeps this rank's own chunk of its input, an
# all-to-all returns its input -- one device copy of the output, the local write traffic the real
# collective has too.
_FAKE = int(os.environ.get("DTG_FAKE_WORLD", "0") or 0) > 1


def fake_fill_scatter(out: torch.Tensor, x: torch.Tensor, group=None) -> None:
    if _FAKE and backend_of(group) == "fake":
        n, r = world(group), rank(group)
        out.view(-1).copy_(x.reshape(n, -1)[r])


def _xgmi_for(group, x: torch.Tensor, nbytes: int):
    c = _XGMI.get(group)
    if c is not None and x.is_cuda and x.dtype in (torch.bfloat16, torch.float32) and c.fits(nbytes):
        return c
    return None


def all_gather_dim0(x: torch.Tensor, group=None) -> torch.Tensor:
    n = world(group)
    if n == 1:
        return x
    out = torch.empty((x.shape[0] * n,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    c = _xgmi_for(group, x, x.numel() * x.element_size())
    if c is not None:
        return c.all_gather_into(out, x)
    dist.all_gather_into_tensor(out, x, group=group)
    return out


def all_reduce_(x: torch.Tensor, group=None) -> torch.Tensor:
    """In-place sum all-reduce (one-shot xGMI for small TP messages when registered)."""
    if world(group) == 1:
        return x
    c = _xgmi_for(group, x, x.numel() * x.element_size())
    if c is not None and x.is_contiguous():
        return c.all_reduce_(x)
    dist.all_reduce(x, group=group)
    return x


def reduce_scatter_dim0(x: torch.Tensor, group=None) -> torch.Tensor:
    n = world(group)
    if n == 1:
        return x
    assert x.shape[0] % n == 0, f"dim 0 ({x.shape[0]}) must divide by group size {n}"
    chunk = x.shape[0] // n
    if backend_of(group) == "gloo":
        y = x.clone()
        dist.all_reduce(y, group=group)
        r = rank(group)
        return y[r * chunk:(r + 1) * chunk].contiguous()
    out = torch.empty((chunk,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    c = _xgmi_for(group, x, x.numel() * x.element_size())
    if c is not None:
        c.reduce_scatter_into(out, x)
        c.release_slot(x, None)  # stream-ordered: the slot is free for the next producer
        return out
    dist.reduce_scatter_tensor(out, x, group=group)
    fake_fill_scatter(out, x, group)
    return out


def all_to_all_dim0(x: torch.Tensor, group=None) -> torch.Tensor:
    """x [n * c, ...]: chunk j goes to rank j; returns [n * c, ...] whose chunk i came from rank i.

    RCCL runs it as one all-to-all (every pair of MI355X GPUs in a node has its own xGMI link,
    so the n-1 peer transfers proceed in parallel).  gloo with device tensors (the 1-GPU test
    rehearsals) is emulated by an all-gather and a local pick."""
    n = world(group)
    if n == 1:
        return x
    assert x.shape[0] % n == 0, f"dim 0 ({x.shape[0]}) must divide by group size {n}"
    x = x.contiguous()
    if backend_of(group) == "gloo" and x.is_cuda:
        c = x.shape[0] // n
        r = rank(group)
        full = all_gather_dim0(x, group).view(n, n, c, *x.shape[1:])  # [src, dst, c, ...]
        return full[:, r].reshape(x.shape).contiguous()
    out = torch.empty_like(x)
    dist.all_to_all_single(out, x, group=group)
    if _FAKE and backend_of(group) == "fake":
        out.copy_(x)
    return out


def all_gather_stack_async(x: torch.Tensor, group=None):
    """(out [n, *x.shape], work): every rank's x stacked rank-major, issued asynchronously on
    RCCL (work.wait() orders the current stream behind it); gloo runs it synchronously."""
    n = world(group)
    out = torch.empty((n,) + tuple(x.shape), dtype=x.dtype, device=x.device)
    if n == 1:
        out[0].copy_(x)
        return out, _DoneWork()
    x = x.contiguous()
    c = _xgmi_for(group, x, x.numel() * x.element_size())
    if c is not None:  # direct-peer library on a side stream (latency-bound message)
        return out, _on_side_stream(lambda: c.all_gather_into(out.view(-1), x.view(-1)), out, x)
    if backend_of(group) == "gloo":
        dist.all_gather(list(out.unbind(0)), x, group=group)
        return out, _DoneWork()
    work = dist.all_gather_into_tensor(out, x, group=group, async_op=True)
    return out, work


def all_gather_into(out: torch.Tensor, shard: torch.Tensor, group=None, async_op=False):
    """Flat all-gather: out.numel() == shard.numel() * world."""
    work = dist.all_gather_into_tensor(out, shard, group=group, async_op=async_op)
    return work


class _DoneWork:
    def wait(self):
        return True

    def is_completed(self):
        return True


def reduce_scatter_into(out: torch.Tensor, full: torch.Tensor, group=None, async_op=False):
    """Flat sum reduce-scatter of `full` into this rank's `out` chunk."""
    if backend_of(group) == "gloo":
        dist.all_reduce(full, group=group)
        r = rank(group)
        n = out.numel()
        out.copy_(full.view(-1)[r * n:(r + 1) * n].view_as(out))
        return _DoneWork() if async_op else None
    work = dist.reduce_scatter_tensor(out, full, group=group, async_op=async_op)
    fake_fill_scatter(out, full, group)
    return work


# ------------------------------------------------------------------------------------------------
# Asynchronous dim-0 gather / scatter for the overlapped tensor-parallel regions
# (parallel/async_tp.py).  Each returns a work object whose wait() makes the CURRENT stream wait
# for the result (RCCL: the PG's own stream; xGMI: a side stream of this module), so compute
# issued between the call and wait() overlaps the transfer.
# ------------------------------------------------------------------------------------------------
_SIDE = {}


def _side_stream(device):
    s = _SIDE.get(device.index)
    if s is None:
        s = _SIDE[device.index] = torch.cuda.Stream(device=device)
    return s


class _StreamWork:
    def __init__(self, event, device):
        self.event, self.device = event, device

    def wait(self):
        torch.cuda.current_stream(self.device).wait_event(self.event)
        return True

    def is_completed(self):
        return self.event.query()


def _on_side_stream(fn, *tensors):
    dev = tensors[0].device
    cur = torch.cuda.current_stream(dev)
    side = _side_stream(dev)
    side.wait_stream(cur)
    with torch.cuda.stream(side):
        fn()
    for t in tensors:  # the caching allocator must not hand these out before the side stream is done
        t.record_stream(side)
    ev = torch.cuda.Event()
    ev.record(side)
    return _StreamWork(ev, dev)


def all_gather_dim0_into_async(out: torch.Tensor, x: torch.Tensor, group=None):
    """out [n * c, ...] <- the c-row x of every rank, rank-major."""
    if world(group) == 1:
        out.copy_(x)
        return _DoneWork()
    c = _xgmi_for(group, x, x.numel() * x.element_size())
    if c is not None:
        return _on_side_stream(lambda: c.all_gather_into(out, x), out, x)
    if backend_of(group) == "gloo":
        dist.all_gather_into_tensor(out, x, group=group)
        return _DoneWork()
    work = dist.all_gather_into_tensor(out, x, group=group, async_op=True)
    return work


def reduce_scatter_dim0_into_async(out: torch.Tensor, x: torch.Tensor, group=None):
    """out [c, ...] <- sum over ranks of rows [rank * c, (rank + 1) * c) of x [n * c, ...].
    `x` is not modified."""
    n = world(group)
    if n == 1:
        out.copy_(x)
        return _DoneWork()
    c = _xgmi_for(group, x, x.numel() * x.element_size())
    if c is not None:
        w = _on_side_stream(lambda: c.reduce_scatter_into(out, x), out, x)
        c.release_slot(x, w.event)
        return w
    if backend_of(group) == "gloo":
        y = x.clone()
        dist.all_reduce(y, group=group)
        r, rows = rank(group), out.shape[0]
        out.copy_(y[r * rows:(r + 1) * rows])
        return _DoneWork()
    work = dist.reduce_scatter_tensor(out, x, group=group, async_op=True)
    fake_fill_scatter(out, x, group)
    return work
