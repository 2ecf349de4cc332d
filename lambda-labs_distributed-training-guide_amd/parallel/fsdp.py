"""Fully-sharded data parallel (ZeRO-3) engine over flat per-unit buffers.

Design (MI355X-first, not a wrapper around torch FSDP):
  * A *unit* is a group of modules whose parameters are gathered together: one per decoder
    layer (`policy="transformer"`, the 405B chapter's transformer wrap + Embedding), or greedy
    post-order groups of >= `min_num_params` (`policy="size"`, the `--numel-to-wrap` policy of
    chapter 04).  Everything else belongs to the root unit.
  * Each unit owns one flat bf16 buffer laid out like `FlatSpace` (padded to world*16), so its
    all-gather is ONE `all_gather_into_tensor` (RCCL) into a full buffer whose storage is
    resized to 0 after use (saved autograd views stay valid: the same storage is refilled by
    the next gather); its gradient reduce-scatter is ONE `reduce_scatter_tensor`.
  * Forward: pre-hook waits for the unit's gather, then prefetches the next unit's gather
    (overlaps with compute); post-hook reshards (`reshard_after_forward`) and inserts a
    pre-backward node on the outputs.  Backward: that node re-gathers the unit and prefetches
    the previous one; once every parameter gradient of the unit is written (notification from
    the kernels' gradient routing) the unit's reduce-scatter is launched asynchronously.
  * All shards live in one flat "shard space" per rank: the fused AdamW runs once over it.
  * Sharding for 288 GB HBM3E: default keeps params resharded after forward (ZeRO-3); with
    `reshard_after_forward=False` the gathered units stay resident until backward (ZeRO-2-like
    traffic, 2/3 of the all-gathers) when memory allows.
  * `cpu_offload=True` keeps parameter shards, gradient shards and optimizer state in pinned
    host memory and runs the native C++ AdamW on the CPU (chapter 05).  With
    `overlap_cpu_step` (default) the host update of each unit starts on a worker thread as soon
    as that unit's gradient shard has landed in host memory during the last micro-batch's
    backward, so the CPU optimizer runs under the rest of the backward instead of after it
    (same kernel, same inputs: bit-identical to the post-backward update).
  * Meta-device init: units are materialised one at a time on the GPU, initialised with the
    same seed on every rank, and only the local shard is kept (peak = one unit).
"""
from __future__ import annotations

import contextlib
import math
import time
from collections import deque
from typing import Callable, Dict, Iterable, List, Optional, Sequence

import torch
import torch.distributed as dist
import torch.nn as nn

from ..ops.adamw import adamw_step
from ..ops.grad_routing import reset_grad_state, set_direct_loss_grad
from ..utils import comm

ALIGN = 16


def _round_up(x, m):
    return (x + m - 1) // m * m


def transformer_units(model: nn.Module) -> List[nn.Module]:
    """One unit per decoder layer (the reference's transformer wrap policy); the embedding,
    final norm and lm_head form the root unit, gathered for the whole step (they are needed at
    both ends of forward and backward, so a separate embedding unit would only be re-gathered)."""
    return list(model.layers)


def _callable_unit(m: nn.Module) -> bool:
    # parameter holders (models.llama.Weight) and containers (ModuleList/ModuleDict) are never
    # called, so forward hooks cannot gather them: their parameters belong to the enclosing unit.
    return not getattr(m, "_dtg_param_holder", False) and not isinstance(m, (nn.ModuleList, nn.ModuleDict))


def size_based_units(model: nn.Module, min_num_params: int) -> List[nn.Module]:
    """Post-order greedy wrap like torch's size_based_auto_wrap_policy: a module becomes a unit
    when its not-yet-wrapped parameters number >= min_num_params."""
    units: List[nn.Module] = []
    wrapped = set()

    def visit(m: nn.Module) -> int:
        n = 0
        for c in m.children():
            n += visit(c)
        own = sum(p.numel() for p in m.parameters(recurse=False) if id(p) not in wrapped)
        n += own
        if m is not model and n >= min_num_params and _callable_unit(m):
            units.append(m)
            for p in m.parameters():
                wrapped.add(id(p))
            return 0
        return n

    visit(model)
    return units


class _Unit:
    def __init__(self, engine: "FullyShard", idx: int, module: nn.Module, named: Sequence, is_root: bool):
        self.engine, self.idx, self.module, self.is_root = engine, idx, module, is_root
        # TP-replicated (sequence-parallel) parameters last and contiguous: one TP all-reduce
        # of that slice per unit before its reduce-scatter, instead of one per parameter
        named = [x for x in named if not getattr(x[1], "_dtg_sequence_parallel", False)] + \
                [x for x in named if getattr(x[1], "_dtg_sequence_parallel", False)]
        self.n_sp = sum(1 for _, p in named if getattr(p, "_dtg_sequence_parallel", False))
        self.names = [n for n, _ in named]
        self.params_src = [p for _, p in named]
        self.shapes = [tuple(p.shape) for p in self.params_src]
        W = engine.world
        offs, cur = [], 0
        for p in self.params_src:
            offs.append(cur)
            cur += _round_up(p.numel(), ALIGN)
        self.offsets = offs
        self.numel = _round_up(max(cur, 1), W * ALIGN)
        self.shard_numel = self.numel // W
        self.expected = sum(getattr(p, "_dtg_uses", 1) for p in self.params_src)
        self.pending = self.expected
        self.full: Optional[torch.Tensor] = None  # full param buffer (storage resized to 0 when sharded)
        self.gathered = False
        self.gather_work = None
        self.full_grad: Optional[torch.Tensor] = None
        self.params: List[nn.Parameter] = []
        self.in_backward = False
        self.rs_launched = False


class _PreBackward(torch.autograd.Function):
    @staticmethod
    def forward(ctx, unit, *xs):
        ctx.unit = unit
        ys = tuple(x.view_as(x) for x in xs)
        return ys if len(ys) > 1 else ys[0]

    @staticmethod
    def backward(ctx, *gs):
        ctx.unit.engine._pre_backward(ctx.unit)
        return (None,) + gs


class FullyShard:
    def __init__(self, model: nn.Module, group=None, policy: str = "transformer", min_num_params: int = 100_000_000,
                 device=None, reshard_after_forward: bool = True, cpu_offload: bool = False,
                 state_dtype=torch.bfloat16, init_fn: Optional[Callable] = None, seed: int = 0,
                 prefetch: bool = True, max_inflight_rs: int = 2, tp_group=None, replicate_group=None,
                 overlap_cpu_step: bool = True, force_collectives: bool = False, offload_params: bool = True,
                 grad_ring: int = 0, dp_comm: str = "rccl"):
        self.module = model
        self.group = group
        # HYBRID_SHARD (ZeRO++-style): shard inside `group` (one node's xGMI island), replicate
        # across `replicate_group` (same local rank on every node); each unit's gradient shard is
        # summed over the replicas right after its reduce-scatter, inside the backward (the
        # all-reduce is stream-ordered behind the reduce-scatter and overlaps later units'
        # backward compute), so step() has no exposed collective.
        self.replicate_group = replicate_group
        self.replicas = comm.world(replicate_group) if (replicate_group is not None and dist.is_initialized()) else 1
        self.tp_group = tp_group  # 2-D: sequence-parallel (replicated) grads are summed over TP first
        self.world = comm.world(group) if dist.is_initialized() else 1
        self.rank = comm.rank(group) if self.world > 1 else 0
        self.mode = "fsdp" if self.replicas == 1 else "hybrid"
        # collectives even at world 1 (RCCL rehearsal of the multi-GPU path on one GPU)
        self._coll = self.world > 1 or (force_collectives and dist.is_initialized())
        self.reshard_after_forward = reshard_after_forward
        self.cpu_offload = cpu_offload
        # offload_params=False (ZeRO-Offload layout, the MI355X default in chapter 05 when it fits):
        # the bf16 parameter shard stays resident in HBM as well; gradients and AdamW state live
        # on the host, the host update writes a pinned master copy, and each updated unit shard is
        # copied back on a side stream while the rest of the backward / host update runs.  Per step
        # that is one D2H of gradients and one H2D of parameters instead of two H2D parameter passes
        # (forward and backward gathers) plus the D2H -- and the forward reads HBM only.
        self.offload_params = bool(cpu_offload and offload_params)
        self.resident = bool(cpu_offload and not offload_params)
        self.overlap_cpu_step = overlap_cpu_step
        self._hparams = None  # bound by FlatAdamW: () -> (lr, beta1, beta2, eps, weight_decay)
        self._in_no_sync = False
        self._bwd_step = None  # (step, grad_scale, hparams) while a backward updates units in flight
        self._cpu_pool = None
        self._cpu_futs = []
        self._bwd_stepped = False
        self._bwd_snapshot = None
        self._poisoned = False
        self.prefetch = prefetch
        self.max_inflight_rs = max_inflight_rs
        p0 = next(model.parameters())
        self.dtype = p0.dtype if p0.dtype.is_floating_point else torch.bfloat16
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
        self.device = torch.device(device)
        # ---- units
        mods = transformer_units(model) if policy == "transformer" else size_based_units(model, min_num_params)
        seen = set()
        unit_named = []
        qual = {id(p): n for n, p in model.named_parameters()}
        for m in mods:
            named = [(qual[id(p)], p) for _, p in m.named_parameters() if id(p) not in seen and p.requires_grad]
            for _, p in named:
                seen.add(id(p))
            if named:
                unit_named.append((m, named))
        root_named = [(n, p) for n, p in model.named_parameters() if id(p) not in seen and p.requires_grad]
        self.units: List[_Unit] = []
        for i, (m, named) in enumerate(unit_named):
            self.units.append(_Unit(self, i, m, named, False))
        self.root = _Unit(self, len(self.units), model, root_named, True) if root_named else None
        all_units = self.units + ([self.root] if self.root is not None else [])
        # ---- one shard space for all units (single fused AdamW launch)
        total = sum(u.shard_numel for u in all_units)
        home = torch.device("cpu") if cpu_offload else self.device
        pin = cpu_offload and torch.cuda.is_available()
        # grad_ring=K (CPU offload with the overlapped host step): no host gradient shard for the
        # whole model -- each unit's reduced gradient lands in one of K unit-sized pinned slots,
        # the host AdamW of that unit consumes it, and the slot is reused.  Saves 2 B per
        # parameter of host RAM (101 GB per rank for Llama-3.1-405B at W = 8: the difference
        # between fitting eight ranks' offloaded state in one node's 3 TB or not).
        self.grad_ring = int(grad_ring) if cpu_offload else 0
        # dp_comm="xgmi-dma": unit all-gathers / reduce-scatters as copy-engine pulls between the
        # ranks' shared shard buffers and gradient pools over xGMI (parallel/xgmi_dp.py; one node)
        self.xdp = None
        if (dp_comm == "xgmi-dma" and self._coll and self.world > 1 and self.device.type == "cuda"
                and (not cpu_offload or self.resident)):
            from .xgmi_dp import XgmiFsdp

            self.xdp = XgmiFsdp(group, self.device, nslots=max_inflight_rs + 3)  # + root + current + 1 spare
        self.dp_comm = "xgmi-dma" if self.xdp is not None else "rccl"
        if self.xdp is not None and not cpu_offload:
            self.shard_params = self.xdp.alloc_shards(total, self.dtype)
            self.shard_grads = torch.zeros(total, dtype=self.dtype, device=home)
        elif pin:  # exact-size page-locked buffers (the caching host allocator rounds to 2^k)
            from ..utils.pinned import pinned_zeros

            self.shard_params = pinned_zeros(total, self.dtype)
            self.shard_grads = pinned_zeros(total if not self.grad_ring else 0, self.dtype)
        else:
            self.shard_params = torch.zeros(total, dtype=self.dtype, device=home)
            self.shard_grads = torch.zeros(total if not self.grad_ring else 0, dtype=self.dtype, device=home)
        self.exp_avg = torch.zeros(total, dtype=state_dtype, device=home)
        self.exp_avg_sq = torch.zeros(total, dtype=state_dtype, device=home)
        # resident mode: the GPU copy every gather reads (the host shard_params is the master)
        self.gpu_params = None
        if self.resident:
            self.gpu_params = (self.xdp.alloc_shards(total, self.dtype) if self.xdp is not None
                               else torch.zeros(total, dtype=self.dtype, device=self.device))
        self._h2d_stream = torch.cuda.Stream(device=self.device) if (self.resident and self.device.type == "cuda") else None
        self._d2h_stream = torch.cuda.Stream(device=self.device) if (cpu_offload and self.device.type == "cuda") else None
        self._d2h_events = []
        # offload traffic / host-update accounting (offload_stats): timed copies and updates
        self._xfer = {"d2h": [], "h2d": []}  # (start event, end event, bytes)
        self._host_upd = [0.0, 0]  # seconds in host AdamW, parameters updated
        self._stat_steps = 0
        o = 0
        for u in all_units:
            u.shard_off = o
            o += u.shard_numel
        self.all_units = all_units
        if self.xdp is not None:
            self.xdp.alloc_grad_pool(max(u.numel for u in all_units), self.dtype)
        self._ring, self._ring_busy, self._ring_next = [], [], 0
        if self.grad_ring:
            from ..utils.pinned import pinned_zeros

            slot = max(u.shard_numel for u in all_units)
            self._ring = [pinned_zeros(slot, self.dtype) if pin else torch.zeros(slot, dtype=self.dtype)
                          for _ in range(self.grad_ring)]
            self._ring_busy = [None] * self.grad_ring
        # ---- materialise params: full buffers per unit, shard extraction, param rebinding
        where = {}
        for mn, mm in model.named_modules():
            for pn, p in mm._parameters.items():
                if p is not None:
                    where.setdefault(id(p), []).append((mm, pn))
        init_fn = init_fn or getattr(model, "init_param", None) or _default_init(model)
        # 2-D (FSDP x TP): each TP rank initialises its own slice of every sharded matrix, so the
        # per-parameter seed is offset by the TP rank (see LlamaForCausalLM.init_weights)
        tp_off = 0
        if tp_group is not None and comm.world(tp_group) > 1:
            from ..models.llama import tp_seed_offset

            tp_off = tp_seed_offset(comm.rank(tp_group))
        for u in all_units:
            full = torch.zeros(u.numel, dtype=self.dtype, device=self.device)
            u.full = full
            new = []
            for i, src in enumerate(u.params_src):
                n = math.prod(u.shapes[i])
                view = full[u.offsets[i]:u.offsets[i] + n].view(u.shapes[i])
                if src.device.type == "meta":
                    torch.manual_seed(seed + 7919 * u.idx + i + tp_off)
                    init_fn(u.names[i], view)
                else:
                    with torch.no_grad():
                        view.copy_(src.detach())
                np_ = nn.Parameter(view, requires_grad=src.requires_grad)
                for attr in ("_dtg_sequence_parallel", "_dtg_uses"):
                    if hasattr(src, attr):
                        setattr(np_, attr, getattr(src, attr))
                np_._dtg_unit = u
                np_._dtg_notify = self._on_grad
                np_.register_post_accumulate_grad_hook(_post_accumulate)
                for mm, pn in where.get(id(src), []):
                    mm._parameters[pn] = np_
                new.append(np_)
            u.params = new
            if self._coll and all(p.device.type != "meta" for p in u.params_src):
                # identical init on every rank is assumed; keep rank 0 authoritative (sync_module_states)
                dist.broadcast(full, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
            my = full[self.rank * u.shard_numel:(self.rank + 1) * u.shard_numel]
            self.shard_params[u.shard_off:u.shard_off + u.shard_numel].copy_(my)
            u.params_src = None
            self._free_full(u)
        if self.resident:
            self.gpu_params.copy_(self.shard_params)
        # ---- hooks
        for u in self.units:
            u.module.register_forward_pre_hook(self._make_pre_forward(u))
            u.module.register_forward_hook(self._make_post_forward(u))
        model.register_forward_pre_hook(self._root_pre_forward)
        if self.root is not None:
            model.register_forward_hook(self._root_post_forward)
        self._rs_inflight = deque()
        self._order: List[_Unit] = []  # forward execution order (recorded on the first step)
        self._record_order = True
        self.step_count = 0
        self.accum_count = 0
        self._sync_enabled = True
        self._first_micro = True
        self._final_micro = None  # set by backward(); None = derive from no_sync() (external callers)
        set_direct_loss_grad(True)

    # ------------------------------------------------------------------ memory helpers
    def _shard_view(self, u: _Unit, buf: torch.Tensor) -> torch.Tensor:
        return buf[u.shard_off:u.shard_off + u.shard_numel]

    def _free_full(self, u: _Unit):
        if u.full is not None and u.full.untyped_storage().size() > 0:
            u.full.untyped_storage().resize_(0)
        u.gathered = False

    def _alloc_full(self, u: _Unit):
        st = u.full.untyped_storage()
        if st.size() == 0:
            st.resize_(u.numel * u.full.element_size())

    # ------------------------------------------------------------------ gather / reshard
    def _issue_gather(self, u: _Unit):
        if u.gathered or u.gather_work is not None:
            return
        self._alloc_full(u)
        if self.resident:
            ev = getattr(u, "h2d_event", None)
            if ev is not None:  # the updated shard's copy back from the host update
                torch.cuda.current_stream(self.device).wait_event(ev)
                u.h2d_event = None
            shard = self._shard_view(u, self.gpu_params)
        else:
            shard = self._shard_view(u, self.shard_params)
        if self.cpu_offload and not self.resident:
            shard = shard.to(self.device, non_blocking=True)
        with torch.autograd._unsafe_preserve_version_counter(u.full):
            if not self._coll:
                u.full.copy_(shard)
                u.gather_work = None
                u.gathered = True
                return
            if self.xdp is not None:
                u.gather_work = self.xdp.gather(u.full, u.shard_off, u.shard_numel, shard)
                u._gather_src = shard
                return
            if comm.backend_of(self.group) == "gloo":
                dist.all_gather_into_tensor(u.full, shard.contiguous(), group=self.group)
                u.gathered = True
                return
            u.gather_work = dist.all_gather_into_tensor(u.full, shard, group=self.group, async_op=True)
        u._gather_src = shard  # keep the (H2D) source alive until the gather completes

    def _wait_gather(self, u: _Unit):
        self._issue_gather(u)
        if u.gather_work is not None:
            u.gather_work.wait()
            u.gather_work = None
            u.gathered = True
        u._gather_src = None

    def _reshard(self, u: _Unit):
        if u.gather_work is not None:
            u.gather_work.wait()
            u.gather_work = None
        self._free_full(u)

    # ------------------------------------------------------------------ forward hooks
    def _root_pre_forward(self, module, args, kwargs=None):
        if self.root is not None:
            self._wait_gather(self.root)
            self.root.in_backward = False
            if torch.is_grad_enabled():
                self._prepare_grads(self.root)
        if self.prefetch and self._order and not self._record_order:
            self._issue_gather(self._order[0])

    def _root_post_forward(self, module, args, out):
        self._record_order = False
        return out

    def _make_pre_forward(self, u: _Unit):
        def hook(module, args):
            self._wait_gather(u)
            if u.in_backward:  # activation-checkpoint recompute inside backward
                return None
            if self._record_order:
                self._order.append(u)
            elif self.prefetch:
                k = self._order.index(u) if u in self._order else -1
                if 0 <= k < len(self._order) - 1:
                    self._issue_gather(self._order[k + 1])
            return None

        return hook

    def _make_post_forward(self, u: _Unit):
        def hook(module, args, out):
            if u.in_backward or not torch.is_grad_enabled():
                return out
            if self.reshard_after_forward:
                self._reshard(u)
            flat, rebuild = _flatten_out(out)
            if not any(t.requires_grad for t in flat):
                return out
            new = _PreBackward.apply(u, *flat)
            new = new if isinstance(new, tuple) else (new,)
            return rebuild(list(new))

        return hook

    # ------------------------------------------------------------------ backward
    def _pre_backward(self, u: _Unit):
        if u.in_backward:
            return
        u.in_backward = True
        self._wait_gather(u)
        self._prepare_grads(u)
        if self.prefetch and u in self._order:
            k = self._order.index(u)
            if k > 0:
                self._issue_gather(self._order[k - 1])

    def _prepare_grads(self, u: _Unit):
        if u.full_grad is not None:
            return
        if self.xdp is not None:  # a slot of the shared gradient pool the peers pull from
            u.full_grad, u.grad_slot = self.xdp.grad_buffer(u.numel)
        else:
            u.full_grad = torch.empty(u.numel, dtype=self.dtype, device=self.device)
        # a fresh (uninitialised) full gradient per micro-batch: the first write of every param
        # must overwrite, not accumulate (micro-batches are summed in the gradient shard)
        reset_grad_state(u.params)
        for i, p in enumerate(u.params):
            n = math.prod(u.shapes[i])
            p.main_grad = u.full_grad[u.offsets[i]:u.offsets[i] + n].view(u.shapes[i])
        u.pending = u.expected
        u.rs_launched = False

    def _on_grad(self, p):
        u = p._dtg_unit
        u.pending -= 1
        if u.pending == 0:
            self._launch_rs(u)

    def _launch_rs(self, u: _Unit):
        if u.rs_launched:
            return
        u.rs_launched = True
        # zero the padding / never-written params so the reduce-scatter sums only real grads
        for i, p in enumerate(u.params):
            if not getattr(p, "_dtg_grad_written", False):
                p.main_grad.zero_()
        end = u.offsets[-1] + math.prod(u.shapes[-1]) if u.params else 0
        if end < u.numel:
            u.full_grad[end:].zero_()
        if u.n_sp and self.tp_group is not None and comm.world(self.tp_group) > 1:
            lo = u.offsets[len(u.params) - u.n_sp]
            comm.all_reduce_(u.full_grad[lo:end], self.tp_group)
        gs = self._shard_view(u, self.shard_grads)
        first = self._first_micro
        direct = not (self.cpu_offload or not first)  # reduce-scatter straight into the grad shard
        out = gs if direct else torch.empty(u.shard_numel, dtype=self.dtype, device=self.device)
        if not self._coll:
            out.copy_(u.full_grad)
            work = None
        elif self.xdp is not None:
            work = self.xdp.reduce_scatter(u.grad_slot, u.shard_numel, out)
        else:
            work = comm.reduce_scatter_into(out, u.full_grad, group=self.group, async_op=True)
        self._rs_inflight.append((u, work, out, first, direct))
        if not u.is_root and self.reshard_after_forward:
            self._reshard(u)
        while len(self._rs_inflight) > self.max_inflight_rs:
            self._complete_rs(*self._rs_inflight.popleft())

    def _complete_rs(self, u, work, out, first, direct):
        if work is not None:
            work.wait()
        merged = False
        final = (not self._in_no_sync) if self._final_micro is None else self._final_micro
        if self.replicas > 1 and final:
            # HYBRID: the shard summed over the replicas once per optimizer step, on the last
            # micro-batch: earlier micro-batches accumulate locally (no inter-replica traffic)
            # and their sum joins this micro-batch's shard before the one all-reduce.  RCCL:
            # wait() only orders the current stream behind it; the host keeps queueing kernels.
            if not first:
                gs = self._shard_view(u, self.shard_grads)
                if gs.device.type == "cpu":
                    self._sync_d2h()
                    out.add_(gs.to(out.device, non_blocking=False))
                else:
                    out.add_(gs)
                merged = True
            ar = dist.all_reduce(out, group=self.replicate_group, async_op=True)
            ar.wait()
        ev = None
        gsrc = None
        if not direct:
            gs = self._ring_slot(u) if self.grad_ring else self._shard_view(u, self.shard_grads)
            gsrc = gs
            if (first or merged) and self._d2h_stream is not None and gs.device.type == "cpu":
                # offload: the gradient shard goes to pinned host memory on a side stream, so the
                # host thread keeps queueing backward kernels; the host update (or step()) waits
                # for the copy's event
                cur = torch.cuda.current_stream(self.device)
                self._d2h_stream.wait_stream(cur)
                with torch.cuda.stream(self._d2h_stream):
                    t0 = torch.cuda.Event(enable_timing=True)
                    t0.record(self._d2h_stream)
                    gs.copy_(out, non_blocking=True)
                    ev = torch.cuda.Event(enable_timing=True)
                    ev.record(self._d2h_stream)
                self._xfer_add("d2h", t0, ev, out.numel() * out.element_size())
                out.record_stream(self._d2h_stream)
                self._d2h_events.append(ev)
            elif first or merged:
                gs.copy_(out)
            else:
                self._sync_d2h()  # the previous micro-batch's copy into gs must have landed
                gs.add_(out.to(gs.device))
        if self._bwd_step is not None:
            self._submit_host_step(u, ev, gsrc)
        u.full_grad = None
        for p in u.params:
            p.main_grad = None

    def finish_grad_sync(self):
        for u in self.all_units:
            if u.full_grad is not None and not u.rs_launched:
                self._launch_rs(u)
        while self._rs_inflight:
            self._complete_rs(*self._rs_inflight.popleft())
        # every unit is resharded: the optimizer updates the shards, so a full buffer kept from
        # this step would be stale in the next forward
        for u in self.all_units:
            u.in_backward = False
            self._reshard(u)
        self._first_micro = False

    @contextlib.contextmanager
    def no_sync(self):
        """Gradient accumulation: FSDP still reduce-scatters each micro-batch (memory stays
        sharded) and accumulates into the gradient shard; inside this context a backward is
        known not to be the last micro-batch (no host optimizer overlap)."""
        prev, self._in_no_sync = self._in_no_sync, True
        try:
            yield
        finally:
            self._in_no_sync = prev

    def _sync_d2h(self):
        evs, self._d2h_events = self._d2h_events, []
        for ev in evs:
            ev.synchronize()

    def _ring_slot(self, u):
        """Next gradient staging slot (grad_ring), once the host update that last read it is done."""
        k = self._ring_next
        self._ring_next = (k + 1) % len(self._ring)
        fut = self._ring_busy[k]
        if fut is not None:
            fut.result()  # normally long finished: the host update keeps pace with the backward
            self._ring_busy[k] = None
        self._ring_k = k
        return self._ring[k][:u.shard_numel]

    def _submit_host_step(self, u, ev=None, grad=None):
        import concurrent.futures as cf

        from ..ops.adamw import adamw_step_cpu

        if self._cpu_pool is None:  # one worker: units update in order, OpenMP inside the kernel
            self._cpu_pool = cf.ThreadPoolExecutor(max_workers=1, thread_name_prefix="dtg-host-adamw")
        step, scale, (lr, b1, b2, eps, wd) = self._bwd_step
        sl = slice(u.shard_off, u.shard_off + u.shard_numel)
        g = grad if (grad is not None and self.grad_ring) else self.shard_grads[sl]

        def update():
            if ev is not None:  # this unit's gradient shard has landed in host memory
                ev.synchronize()
            t0 = time.perf_counter()
            adamw_step_cpu(self.shard_params[sl], g, self.exp_avg[sl], self.exp_avg_sq[sl],
                           lr=lr, step=step, beta1=b1, beta2=b2, eps=eps, weight_decay=wd, grad_scale=scale)
            self._host_upd[0] += time.perf_counter() - t0
            self._host_upd[1] += u.shard_numel
            if self.resident:
                self._copy_back(u, sl)

        fut = self._cpu_pool.submit(update)
        self._cpu_futs.append(fut)
        if self.grad_ring and grad is not None:
            self._ring_busy[self._ring_k] = fut

    def _copy_back(self, u, sl):
        """Resident mode: updated host shard -> its HBM copy on the H2D side stream; the next
        gather of the unit waits for the event (`_issue_gather`)."""
        if self._h2d_stream is None:
            self.gpu_params[sl].copy_(self.shard_params[sl])
            return
        with torch.cuda.device(self.device), torch.cuda.stream(self._h2d_stream):
            t0 = torch.cuda.Event(enable_timing=True)
            t0.record(self._h2d_stream)
            self.gpu_params[sl].copy_(self.shard_params[sl], non_blocking=True)
            ev = torch.cuda.Event(enable_timing=True)
            ev.record(self._h2d_stream)
        self._xfer_add("h2d", t0, ev, (sl.stop - sl.start) * self.gpu_params.element_size())
        u.h2d_event = ev

    def backward(self, loss, last_microbatch: Optional[bool] = None):
        """Backward of one micro-batch.  With CPU offload and `overlap_cpu_step`, the host AdamW
        of each unit runs during the backward that is known to be the last micro-batch of the
        step: `last_microbatch=True`, or None outside `no_sync()`.  Pass False (or use
        `no_sync()`) for earlier micro-batches.  A second backward after an overlapped one
        without step()/zero_grad() in between is an error (it would update twice)."""
        if self._poisoned:
            raise RuntimeError("FullyShard: a previous backward failed after host updates started; "
                               "parameters are partially updated -- reload a checkpoint")
        if self._bwd_stepped:
            raise RuntimeError("FullyShard.backward: the previous backward already applied the optimizer "
                               "update (overlap_cpu_step); call step()/zero_grad() first, or mark earlier "
                               "micro-batches with no_sync() / last_microbatch=False")
        final = (not self._in_no_sync) if last_microbatch is None else bool(last_microbatch)
        self._final_micro = final  # HYBRID: the replica all-reduce runs on the final micro-batch only
        overlap = (self.cpu_offload and self.overlap_cpu_step and self._hparams is not None and final)
        if self.grad_ring and not (overlap and self.accum_count == 0):
            raise RuntimeError("FullyShard(grad_ring=...): the host gradient ring has no whole-model gradient "
                               "shard to accumulate into; it needs the overlapped host step (overlap_cpu_step, a "
                               "bound FlatAdamW) on the only micro-batch of each step (no gradient accumulation)")
        if overlap:  # the last micro-batch: its per-unit gradient shards are final on arrival
            scale = 1.0 / (self.world * self.replicas * (self.accum_count + 1))
            self._bwd_step = (self.step_count + 1, scale, self._hparams())
        ok = False
        try:
            loss.backward()
            self.accum_count += 1
            self.finish_grad_sync()
            ok = True
        finally:
            self._final_micro = None  # a caller driving loss.backward() itself derives it from no_sync()
            snap, self._bwd_step = self._bwd_step, None
            if not ok and self._cpu_futs:
                # host updates of some units were submitted: let them finish, then refuse to
                # step on a half-updated model (a retry would apply AdamW twice to those units)
                try:
                    self._join_host_steps()
                finally:
                    self._poisoned = True
        self._bwd_stepped = overlap
        self._bwd_snapshot = snap if overlap else None

    def _join_host_steps(self):
        futs, self._cpu_futs = self._cpu_futs, []
        for f in futs:
            f.result()
        self._sync_d2h()

    def zero_grad(self):
        self._join_host_steps()  # never let a host update race the next forward's shard reads
        if self._bwd_stepped:
            # the update already ran during backward (a skipped step() still counts as a step)
            self._bwd_stepped = False
            self.step_count += 1
        for u in self.all_units:
            reset_grad_state(u.params)
            u.pending = u.expected
        self.accum_count = 0
        self._first_micro = True

    # ------------------------------------------------------------------ optimizer
    def step(self, lr, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.01, grad_scale=None):
        if self._poisoned:
            raise RuntimeError("FullyShard.step: a failed backward left units partially updated")
        if self.grad_ring and not self._bwd_stepped:
            raise RuntimeError("FullyShard.step: grad_ring engines update during backward only")
        if self._bwd_stepped:  # overlap_cpu_step: every unit was updated during backward
            step, scale, hp = self._bwd_snapshot
            if grad_scale is not None or tuple(hp) != (lr, beta1, beta2, eps, weight_decay):
                raise RuntimeError("FullyShard.step: the update already ran during backward with "
                                   f"{hp} and grad_scale={scale}; step() got different hyper-parameters "
                                   f"{(lr, beta1, beta2, eps, weight_decay)} / grad_scale={grad_scale}. "
                                   "Change them before backward(), or pass overlap_cpu_step=False")
            self.step_count += 1
            self._bwd_stepped = False
            self._join_host_steps()
            return
        self.step_count += 1
        self._sync_d2h()
        if grad_scale is None:
            grad_scale = 1.0 / (self.world * self.replicas * max(1, self.accum_count))
        # (HYBRID: the gradient shards were already summed over the replicas during backward)
        if self.cpu_offload:
            from ..ops.adamw import adamw_step_cpu

            t0 = time.perf_counter()
            adamw_step_cpu(self.shard_params, self.shard_grads, self.exp_avg, self.exp_avg_sq, lr=lr,
                           step=self.step_count, beta1=beta1, beta2=beta2, eps=eps, weight_decay=weight_decay,
                           grad_scale=grad_scale)
            self._host_upd[0] += time.perf_counter() - t0
            self._host_upd[1] += self.shard_params.numel()
            if self.resident:
                self.sync_params_after_load()
        else:
            adamw_step(self.shard_params, self.shard_grads, self.exp_avg, self.exp_avg_sq, lr=lr, step=self.step_count,
                       beta1=beta1, beta2=beta2, eps=eps, weight_decay=weight_decay, grad_scale=grad_scale)

    def _xfer_add(self, kind, t0, t1, nbytes):
        xs = self._xfer[kind]
        xs.append((t0, t1, nbytes))
        if len(xs) > 4096:  # fold resolved copies into a running (ms, bytes) entry: bounded lists
            xs[-1][1].synchronize()
            ms = sum(a.elapsed_time(b) if a is not None else b for a, b, _ in xs)
            self._xfer[kind] = [(None, ms, sum(b for _, _, b in xs))]

    def offload_stats(self, reset: bool = True) -> dict:
        """CPU offload accounting since the last reset, per optimizer step: host AdamW seconds and
        GB/s (14 B per parameter: p, m, v read + written in bf16, g read), gradient D2H and
        parameter H2D GB and GB/s (sum of each copy's own HIP-event time on its side stream).
        Synchronises the copies it reads (call at log time)."""
        steps = max(1, self.step_count - self._stat_steps)
        out = {}
        secs, n = self._host_upd
        if n:
            out["host_adamw_s"] = secs / steps
            out["host_adamw_gbs"] = 14 * n / secs / 1e9 if secs > 0 else 0.0
        for k in ("d2h", "h2d"):
            xs = self._xfer[k]
            if xs:
                if xs[-1][0] is not None:
                    xs[-1][1].synchronize()
                ms = sum(a.elapsed_time(b) if a is not None else b for a, b, _ in xs)
                nbytes = sum(b for _, _, b in xs)
                out[f"{k}_gb"] = nbytes / steps / 1e9
                out[f"{k}_gbs"] = nbytes / (ms / 1e3) / 1e9 if ms > 0 else 0.0
        if reset:
            self._xfer = {"d2h": [], "h2d": []}
            self._host_upd = [0.0, 0]
            self._stat_steps = self.step_count
        return out

    def sync_params_after_load(self):
        """Resident offload: the host master shard changed (checkpoint / pretrained load, a
        post-backward host step) -> refresh the HBM copy the gathers read."""
        if not self.resident:
            return
        for u in self.all_units:
            u.h2d_event = None
            if not u.in_backward:
                self._free_full(u)
        self.gpu_params.copy_(self.shard_params)

    # ------------------------------------------------------------------ state
    def optimizer_state(self):
        return {"step": self.step_count, "exp_avg": self.exp_avg, "exp_avg_sq": self.exp_avg_sq,
                "mode": "fsdp", "world": self.world, "rank": self.rank}

    def load_optimizer_state(self, st):
        assert st["world"] == self.world, "optimizer state layout mismatch"
        self.step_count = int(st["step"])
        self.exp_avg.copy_(st["exp_avg"])
        self.exp_avg_sq.copy_(st["exp_avg_sq"])

    def ckpt_pieces(self):
        """This rank's owned slices: (param_name, start_in_param, numel, param_view, state_index)."""
        out = []
        for u in self.all_units:
            s = self.rank * u.shard_numel
            e = s + u.shard_numel
            for i, name in enumerate(u.names):
                off, n = u.offsets[i], math.prod(u.shapes[i])
                lo, hi = max(off, s), min(off + n, e)
                if lo < hi:
                    k = u.shard_off + (lo - s)
                    out.append((name, lo - off, hi - lo, self.shard_params[k:k + (hi - lo)], k))
        return out

    @torch.no_grad()
    def full_state_dict(self, rank0_only: bool = True) -> Dict[str, torch.Tensor]:
        """Gather every unit and return the full (CPU) state dict, names as in model.state_dict()."""
        out = {}
        qual = {id(p): n for n, p in self.module.named_parameters()}
        for u in self.all_units:
            self._wait_gather(u)
            for p in u.params:
                if (not rank0_only) or self.rank == 0:
                    out[qual[id(p)]] = p.detach().cpu().clone()
            self._reshard(u)
        return out


def _flatten_out(out):
    if isinstance(out, torch.Tensor):
        return [out], lambda xs: xs[0]
    if isinstance(out, tuple) and all(isinstance(t, torch.Tensor) for t in out):
        return list(out), lambda xs: tuple(xs)
    if isinstance(out, tuple):
        idx = [i for i, t in enumerate(out) if isinstance(t, torch.Tensor)]

        def rebuild(xs):
            lst = list(out)
            for i, x in zip(idx, xs):
                lst[i] = x
            return tuple(lst)

        return [out[i] for i in idx], rebuild
    return [], lambda xs: out


def _post_accumulate(p):
    if p.grad is None:
        return
    from ..ops.grad_routing import route_param_grad

    g = p.grad
    p.grad = None
    route_param_grad(p, g)


def _default_init(model):
    cfg = getattr(model, "config", None)
    std = getattr(cfg, "initializer_range", 0.02)

    def init(name, t):
        with torch.no_grad():
            if name.endswith("layernorm.weight") or name.endswith("norm.weight") or ".ln_" in name or name.startswith("ln_"):
                if name.endswith("bias"):
                    t.zero_()
                else:
                    t.fill_(1.0)
            elif name.endswith("bias"):
                t.zero_()
            else:
                t.normal_(0.0, std)

    return init
