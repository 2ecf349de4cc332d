"""Flat parameter / gradient storage with communication buckets.

Every engine (single device, DDP, ZeRO, FSDP units) keeps a rank's trainable parameters in ONE
contiguous bf16 buffer and their gradients in a second one (`param.main_grad` views), laid out
in *backward* order so consecutive gradients fill the same bucket.  Buckets are contiguous,
padded to a multiple of `world * 16` elements, so every bucket maps to exactly one RCCL
all-reduce / reduce-scatter / all-gather on a contiguous slice (no copy-in/copy-out), and the
fused AdamW kernel runs over contiguous shards with 16-byte vector accesses.

Bucket size default is 256 MiB: on MI355X (7 point-to-point xGMI links per GPU) RCCL reaches
its bandwidth plateau only for messages of a few hundred MB, and with 288 GB of HBM3E the extra
buffering costs nothing (the reference's 25 MB DDP default is tuned for NVLink/NVSwitch).
"""
from __future__ import annotations

import math
from typing import Callable, List, Optional, Sequence, Tuple

import torch
import torch.nn as nn

ALIGN = 16  # elements; 32 bytes for bf16, keeps every view 16-B aligned


def _round_up(x, m):
    return (x + m - 1) // m * m


class Bucket:
    __slots__ = ("index", "start", "end", "params", "pending", "expected", "work", "launched", "stepped", "trailing")

    def __init__(self, index, start, end, params, trailing=False):
        self.index, self.start, self.end, self.params = index, start, end, params
        self.trailing = trailing  # the separate last bucket of `trailing`-predicate params
        self.expected = sum(getattr(p, "_dtg_uses", 1) for p in params)
        self.pending = self.expected
        self.work = None
        self.launched = False
        self.stepped = False

    @property
    def numel(self):
        return self.end - self.start


class FlatSpace:
    """Owns the flat param/grad buffers for `named_params` (already materialised tensors)."""

    def __init__(self, named_params: Sequence[Tuple[str, nn.Parameter]], device, world: int = 1,
                 bucket_bytes: int = 256 << 20, dtype=torch.bfloat16, grad_dtype=None, reverse=True,
                 alloc_params=True, trailing: Optional[Callable] = None, alloc: Optional[Callable] = None):
        """`trailing(p)`: parameters moved into one extra bucket after all others (tensor-
        parallel replicated norm weights: their gradients are summed over TP with ONE
        all-reduce of that bucket instead of one per parameter).  `alloc(numel, dtype, kind)`
        (kind "param" | "grad") provides the flat buffers instead of torch.zeros (IPC-shared
        memory for the xGMI copy-engine collectives, parallel/xgmi_dp.py)."""
        self.world = world
        self.device = torch.device(device)
        self.dtype = dtype
        self.grad_dtype = grad_dtype or dtype
        items = list(named_params)
        if reverse:
            items = items[::-1]
        tail = [(n, p) for n, p in items if trailing is not None and trailing(p)]
        items = [(n, p) for n, p in items if not (trailing is not None and trailing(p))] + tail
        n_main = len(items) - len(tail)
        self.names = [n for n, _ in items]
        esz = torch.tensor([], dtype=dtype).element_size()
        cap = max(1, bucket_bytes // esz)
        unit = world * ALIGN
        # Assign offsets; close a bucket when it would exceed `cap`.
        self.offsets: List[int] = []
        buckets_spec = []
        cur_start, cur, cur_params = 0, 0, []
        for k, (n, p) in enumerate(items):
            sz = _round_up(p.numel(), ALIGN)
            if cur_params and ((cur - cur_start) + sz > cap or k == n_main):
                end = cur_start + _round_up(cur - cur_start, unit)
                buckets_spec.append((cur_start, end, cur_params))
                cur_start = cur = end
                cur_params = []
            self.offsets.append(cur)
            cur_params.append(p)
            cur += sz
        if cur_params:
            end = cur_start + _round_up(cur - cur_start, unit)
            buckets_spec.append((cur_start, end, cur_params))
            cur = end
        self.numel = cur
        self.shapes = [tuple(p.shape) for _, p in items]
        self.params_src = [p for _, p in items]
        if alloc is None:
            alloc = lambda n, dt, kind: torch.zeros(n, dtype=dt, device=self.device)  # noqa: E731
        self.param_buf = alloc(self.numel, dtype, "param") if alloc_params else None
        self.grad_buf = alloc(self.numel, self.grad_dtype, "grad")
        self.buckets = [Bucket(i, s, e, ps, trailing=bool(tail) and i == len(buckets_spec) - 1)
                        for i, (s, e, ps) in enumerate(buckets_spec)]
        self.param_bucket = []
        for b in self.buckets:
            self.param_bucket.extend([b] * len(b.params))

    def param_view(self, i: int, buf: Optional[torch.Tensor] = None) -> torch.Tensor:
        buf = self.param_buf if buf is None else buf
        o = self.offsets[i]
        n = math.prod(self.shapes[i])
        return buf[o:o + n].view(self.shapes[i])

    def grad_view(self, i: int) -> torch.Tensor:
        o = self.offsets[i]
        n = math.prod(self.shapes[i])
        return self.grad_buf[o:o + n].view(self.shapes[i])

    def shard_range(self, bucket: Bucket, rank: int) -> Tuple[int, int]:
        n = bucket.numel // self.world
        return bucket.start + rank * n, bucket.start + (rank + 1) * n


def rebind_parameters(module: nn.Module, space: FlatSpace, copy_data: bool = True,
                      notify: Optional[Callable] = None) -> List[nn.Parameter]:
    """Replace every parameter in `space` by a Parameter viewing the flat buffer (data copied),
    attach `main_grad` views and the engine's ready callback.  Returns the new parameters in
    flat (backward) order."""
    where = {}
    for mod_name, mod in module.named_modules():
        for pn, p in mod._parameters.items():
            if p is not None:
                where.setdefault(id(p), []).append((mod, pn))
    new_params = []
    for i, src in enumerate(space.params_src):
        view = space.param_view(i)
        if copy_data and src.device.type != "meta":
            with torch.no_grad():
                view.copy_(src.detach().to(view.dtype))
        np_ = nn.Parameter(view, requires_grad=src.requires_grad)
        for attr in ("_dtg_sequence_parallel", "_dtg_uses", "_dtg_name"):
            if hasattr(src, attr):
                setattr(np_, attr, getattr(src, attr))
        np_.main_grad = space.grad_view(i)
        np_._dtg_bucket = space.param_bucket[i]
        if notify is not None:
            np_._dtg_notify = notify
            # Parameters whose gradient arrives through ordinary autograd (.grad), e.g. ATen
            # LayerNorm in GPT-2: move it into main_grad and fire the same notification.
            np_.register_post_accumulate_grad_hook(_post_accumulate)
        for mod, pn in where.get(id(src), []):
            mod._parameters[pn] = np_
        new_params.append(np_)
    return new_params


def _post_accumulate(p):
    if p.grad is None:
        return
    from ..ops.grad_routing import route_param_grad

    g = p.grad
    p.grad = None
    route_param_grad(p, g)
