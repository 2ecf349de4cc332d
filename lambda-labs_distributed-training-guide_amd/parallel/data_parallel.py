"""Data-parallel engines over flat buckets: single device, DDP, ZeRO.

  mode="single"  world of one: flat buffers + fused AdamW, no communication.
  mode="ddp"     replicated params; each gradient bucket is all-reduced (RCCL, async) the
                 moment its last gradient is written during backward (overlap), averaging
                 folded into AdamW's grad_scale (no divide pass).
  mode="zero"    ZeRO-2: buckets are reduce-SCATTERED instead (half the bytes of an all-reduce
                 per rank), each rank keeps AdamW state only for its 1/W slice of every bucket,
                 and updated slices are all-gathered back into the replicated parameters.
                 The reference's ZeroRedundancyOptimizer (ZeRO-1: all-reduce + broadcast, state
                 not checkpointable) is strictly more traffic; this engine's state is
                 checkpointable (§2.11 #1).

Transposed weights (bf16 on the GPU; `weight_t=True`): hipBLASLt runs the
backward's dX = dY W at TN speed only with a K-contiguous W^T.  Weights change once per step,
so the optimizer kernel (`adamw_t_`) writes W^T of every weight matrix while the updated values
are in registers, into a persistent buffer the Linear backward reads (`ops.functional._wt`),
instead of every backward transposing every weight (one read + one write of W per step: the
read is saved, the write moves into the optimizer).  Staleness is impossible by construction:
the copy is used only while the flat parameter buffer's version counter still equals the value
recorded after the last refresh, so any other write to the weights (a checkpoint or pretrained
load, a manual edit) makes the backward fall back to transposing until the next step.
Under ZeRO a rank updates only its 1/W slice of each bucket, so the copies are rebuilt instead
as each bucket's parameter all-gather lands: one batched transpose launch per bucket
(`transpose_mats_`) on a side stream, under the next forward's GEMMs, and the backward's dX
GEMM waits for its bucket's event (the transposes left the backward's critical path).

`overlap_optimizer=True` moves the AdamW update into backward: the moment a bucket's gradients
are final (and, with DDP/ZeRO, its all-reduce / reduce-scatter has landed) its update runs on a
side HIP stream while backward keeps the matrix cores busy with the remaining layers; under
ZeRO the bucket's parameter all-gather is issued right behind it.  `optimizer.step()` then only
joins the side stream.  Updates are bit-identical to the post-backward step (same kernel, same
hyper-parameters: the LR scheduler has already stepped for this iteration).

Gradient accumulation (`no_sync()`), parameters unused in a step, tensor-parallel replicated
(sequence-parallel) norm weights and tied embeddings are handled.  All engines present a
torch.optim.Optimizer (`FlatAdamW`) so LR schedulers and the reference's loop shape work.
"""
from __future__ import annotations

import contextlib
import os
from typing import Optional

import torch
import torch.distributed as dist
import torch.nn as nn

from ..ops.adamw import adamw_step
from ..ops.grad_routing import reset_grad_state, set_direct_loss_grad
from ..utils import comm
from .flat import FlatSpace, rebind_parameters


class DataParallel:
    def __init__(self, model: nn.Module, mode: str = "ddp", group=None, tp_group=None,
                 bucket_mb: int = 256, broadcast_from_rank0: bool = True, state_dtype=torch.bfloat16,
                 master_weights: bool = False, overlap_param_gather: bool = True,
                 overlap_optimizer: bool = False, grad_divisor: Optional[int] = None,
                 force_collectives: bool = False, weight_t: Optional[bool] = None, dp_comm: str = "rccl"):
        """dp_comm: "rccl" (default; also the inter-node path) or "xgmi-dma": ZeRO's gradient
        reduce-scatter and parameter all-gather as copy-engine pulls between the ranks' shared
        flat buffers over xGMI (parallel/xgmi_dp.py; one node, no CU time in the overlap)."""
        assert mode in ("single", "ddp", "zero")
        assert dp_comm in ("rccl", "xgmi-dma"), dp_comm
        self.module = model
        self.group = group
        self.tp_group = tp_group
        self.world = comm.world(group) if mode != "single" and dist.is_initialized() else 1
        self.rank = comm.rank(group) if self.world > 1 else 0
        # force_collectives: keep ddp/zero (and every RCCL call they make) even in a world of one,
        # so the 1-GPU box exercises the async work objects, stream waits and in-place gathers of
        # the multi-GPU path over a real RCCL communicator (tests/test_engines_rccl_gpu.py).
        force = force_collectives and mode != "single" and dist.is_initialized()
        self.mode = mode if (self.world > 1 or force) else "single"
        dev = next(model.parameters()).device
        named = [(n, p) for n, p in model.named_parameters() if p.requires_grad]
        for n, p in named:
            p._dtg_name = n
        tp_on = tp_group is not None and comm.world(tp_group) > 1
        self.xdp = None
        if dp_comm == "xgmi-dma" and self.mode == "zero" and self.world > 1 and dev.type == "cuda":
            from .xgmi_dp import XgmiZero

            self.xdp = XgmiZero(group, dev)
        self.dp_comm = "xgmi-dma" if self.xdp is not None else "rccl"
        self.space = FlatSpace(named, dev, world=self.world if self.mode == "zero" else 1,
                               bucket_bytes=bucket_mb << 20, dtype=named[0][1].dtype,
                               trailing=(lambda p: getattr(p, "_dtg_sequence_parallel", False)) if tp_on else None,
                               alloc=self.xdp.alloc if self.xdp is not None else None)
        self._sp_bucket = next((b for b in self.space.buckets if b.trailing), None)
        self._sp_reduced = False
        self.params = rebind_parameters(model, self.space, copy_data=True, notify=self._on_grad)
        self._sync_enabled = True
        self._inflight = []
        if self.mode != "single" and broadcast_from_rank0:
            src = dist.get_global_rank(group, 0) if group is not None else 0
            dist.broadcast(self.space.param_buf, src=src, group=group)
        # Optimizer state over what this rank updates.
        if self.mode == "zero":
            self.shard_ranges = [self.space.shard_range(b, self.rank) for b in self.space.buckets]
            self.shard_numel = sum(e - s for s, e in self.shard_ranges)
            self.grad_shard = torch.zeros(self.shard_numel, dtype=self.space.grad_dtype, device=dev)
            offs, o = [], 0
            for s, e in self.shard_ranges:
                offs.append(o)
                o += e - s
            self.shard_offsets = offs
        else:
            self.shard_numel = self.space.numel
        self.exp_avg = torch.zeros(self.shard_numel, dtype=state_dtype, device=dev)
        self.exp_avg_sq = torch.zeros(self.shard_numel, dtype=state_dtype, device=dev)
        self.master = None
        if master_weights:
            self.master = torch.empty(self.shard_numel, dtype=torch.float32, device=dev)
            self._shard_param_copy(self.master)
        self.step_count = 0
        self.accum_count = 0  # micro-batches accumulated since the last step
        # ZeRO: the post-step parameter all-gathers are left in flight and each bucket is waited
        # for just before the first module that reads it runs in the next forward, so they
        # overlap with the embedding/early-layer compute instead of stalling the step.
        self._pending_ag = {}
        self.overlap_param_gather = overlap_param_gather and self.mode == "zero"
        if self.overlap_param_gather:
            self._install_gather_hooks()
        self.overlap_optimizer = overlap_optimizer
        self._hparams = None  # () -> (lr, beta1, beta2, eps, weight_decay); set by FlatAdamW
        self._opt_stream = torch.cuda.Stream(device=dev) if (overlap_optimizer and dev.type == "cuda") else None
        self._bwd_stepped = False
        # device [lr, 1-beta1^t, sqrt(1-beta2^t)] read by AdamW instead of host scalars while a
        # HIP graph of the step is captured / replayed (dtg.train.graph.GraphedStep)
        self.graph_hyper = None
        # gradients are averaged over `grad_divisor` ranks (default: the whole group).  Context
        # parallelism uses the CP degree's complement: each CP rank's loss is already a share of
        # the global mean, so its gradients are summed over CP and averaged over data parallel.
        self.grad_divisor = grad_divisor or self.world
        # The engine owns the loss: backward(loss) uses an implicit gradient of 1 and any
        # scaling goes into AdamW's grad_scale, which lets the loss head write dW in place.
        set_direct_loss_grad(True)
        # persistent W^T copies refreshed by the optimizer kernel (see the module docstring)
        if weight_t is None:
            import os

            weight_t = os.environ.get("DTG_WEIGHT_T", "1") == "1" and dev.type == "cuda"
        self._wt_buf = None
        self._wt_version = -1
        self._wt_stream = None
        self._wt_ready = {}  # zero: bucket -> event after its W^T transposes (side stream)
        if (weight_t and not overlap_optimizer
                and self.space.dtype == torch.bfloat16 and self.space.grad_dtype == torch.bfloat16) or \
                (weight_t and dev.type == "cpu" and not overlap_optimizer):
            self._build_weight_t()

    # ------------------------------------------------------------------ transposed weights
    def _build_weight_t(self):
        import math

        sp = self.space
        # adamw_t_ tile width (64 x TC tiles; DTG_ADAMT_TC = 64 | 128 | 256, read once here).
        # 256: the register-blocked kernel's fastest walk (profiles/r5/transpose/, r6/knobs/)
        self._wt_tc = int(os.environ.get("DTG_ADAMT_TC", "256"))
        rows_desc, slots, toff, tile0 = [], {}, 0, 0
        for i in range(len(sp.names)):
            shape, off = sp.shapes[i], sp.offsets[i]
            n = math.prod(shape)
            if n == 0:
                continue
            if len(shape) == 2 and shape[0] % 8 == 0 and shape[1] % 8 == 0 and min(shape) >= 64:
                rows, cols, t = shape[0], shape[1], toff
                slots[i] = (toff, rows, cols)
                toff += (n + 127) // 128 * 128  # 256-byte aligned copies, like the allocator's
                rows_desc.append([off, rows, cols, t, tile0])
                tile0 += -(-rows // 64) * -(-cols // self._wt_tc)
                continue
            # No W^T (norm weights, a vocabulary that is not a multiple of 8): updated as full
            # [*, TC] rows plus one short row (within the flat buffer's 16-element padding), so
            # every tile is full -- one [1, n] row would leave 63 of a tile's 64 rows idle
            # (a 157k x 3072 embedding took the update from 8 to 16 ms, profiles/r3/s10).
            n8 = (n + 7) // 8 * 8
            full, rem = divmod(n8, self._wt_tc)
            if full:
                rows_desc.append([off, full, self._wt_tc, -1, tile0])
                tile0 += -(-full // 64)
            if rem:
                rows_desc.append([off + full * self._wt_tc, 1, rem, -1, tile0])
                tile0 += 1
        if not slots:
            return
        dev = sp.param_buf.device
        self._wt_mats = torch.tensor(rows_desc, dtype=torch.long, device=dev)
        self._wt_tiles = tile0
        self._wt_buf = torch.empty(toff, dtype=sp.dtype, device=dev)
        if self.mode == "zero":
            # ZeRO updates 1/W of every bucket, so adamw_t_ cannot write whole W^T copies; they
            # are rebuilt per bucket the moment its parameter all-gather lands, by one batched
            # transpose launch on a side stream that runs under the next forward's GEMMs.
            per_b = {}
            for i, (t, rows, cols) in sorted(slots.items()):
                per_b.setdefault(sp.param_bucket[i].index, []).append((sp.offsets[i], rows, cols, t))
            self._wt_bucket_mats = {}
            for b, mats in per_b.items():
                desc, t0 = [], 0
                for off, rows, cols, t in mats:
                    desc.append([off, rows, cols, t, t0])
                    t0 += -(-rows // 64) * -(-cols // 64)
                host = torch.tensor(desc, dtype=torch.long)
                self._wt_bucket_mats[b] = (host.to(dev), host, t0)
            self._wt_valid = {b: False for b in self._wt_bucket_mats}
            if dev.type == "cuda":
                self._wt_stream = torch.cuda.Stream(device=dev)
        self._wt_views = {}
        for i, (o, rows, cols) in slots.items():
            self._wt_views[i] = self._wt_buf[o:o + rows * cols].view(cols, rows)
        index = {id(p): i for i, p in enumerate(self._space_params())}
        for p in self.params:
            i = index.get(id(p))
            if i is not None and i in self._wt_views:
                p._dtg_wt = (self, i)
        self.refresh_weight_t()

    def _space_params(self):
        """Parameters in FlatSpace order (names -> this engine's rebound parameters)."""
        by_name = {getattr(p, "_dtg_name", None): p for p in self.params}
        return [by_name.get(n) for n in self.space.names]

    @torch.no_grad()
    def refresh_weight_t(self):
        """Recompute every W^T from the current weights (init; any load)."""
        if self._wt_buf is None:
            return
        from ..ops import functional as _F

        ps = self._space_params()
        for i, view in self._wt_views.items():
            w = ps[i]
            view.copy_(_F.ops.transpose2d(w) if w.is_cuda else w.t())
        self._wt_version = self.space.param_buf._version
        if self.mode == "zero":
            self._wt_ready.clear()
            for b in self._wt_valid:
                self._wt_valid[b] = True

    def weight_t(self, i):
        """The current W^T of flat parameter i, or None if the weights changed since the last
        refresh (the caller then transposes)."""
        if self._wt_buf is None or self.space.param_buf._version != self._wt_version:
            return None
        if self.mode == "zero":
            b = self.space.param_bucket[i].index
            if not self._wt_valid.get(b, False):
                return None
            ev = self._wt_ready.pop(b, None)
            if ev is not None:  # the side-stream transposes of this bucket
                torch.cuda.current_stream(self.space.param_buf.device).wait_event(ev)
        return self._wt_views.get(i)

    def _transpose_bucket(self, i, work):
        """ZeRO: W^T of bucket i's matrices once its all-gather (`work`) has landed."""
        ent = self._wt_bucket_mats.get(i) if self._wt_buf is not None and self.mode == "zero" else None
        if ent is None:
            return
        mats_dev, mats_host, ntiles = ent
        st = self._wt_stream
        if st is None:  # CPU engine (gloo tests): in order
            if work is not None:
                work.wait()
            torch.ops.dtg.transpose_mats_(self.space.param_buf.data, self._wt_buf, mats_dev, mats_host, ntiles)
        else:
            st.wait_stream(torch.cuda.current_stream(st.device))
            with torch.cuda.stream(st):
                if work is not None:
                    work.wait()  # the side stream waits for the collective, the host does not
                torch.ops.dtg.transpose_mats_(self.space.param_buf.data, self._wt_buf, mats_dev, mats_host, ntiles)
                ev = torch.cuda.Event()
                ev.record(st)
            self._wt_ready[i] = ev
        self._wt_valid[i] = True

    # ------------------------------------------------------------------ grad sync
    @contextlib.contextmanager
    def no_sync(self):
        """Accumulate gradients locally (skip bucket communication) inside this context."""
        prev = self._sync_enabled
        self._sync_enabled = False
        try:
            yield
        finally:
            self._sync_enabled = prev

    def _reduce_sp(self):
        """Sequence-parallel (TP-replicated) norm weights: every TP rank holds a partial gradient;
        ONE all-reduce over the trailing bucket sums them (was one per parameter: 65
        latency-bound collectives per step at 8B).  Linear, so it may run once after several
        accumulated micro-batches."""
        b = self._sp_bucket
        if b is not None and not self._sp_reduced:
            comm.all_reduce_(self.space.grad_buf[b.start:b.end], self.tp_group)
            self._sp_reduced = True

    def _on_grad(self, p):
        if not self._sync_enabled or (self.mode == "single" and not self.overlap_optimizer):
            return
        b = p._dtg_bucket
        b.pending -= 1
        if b.pending == 0:
            self._launch(b)

    def _launch(self, b):
        if b.launched:
            return
        b.launched = True
        if b.trailing:
            self._reduce_sp()
        view = self.space.grad_buf[b.start:b.end]
        if self.mode == "ddp":
            b.work = dist.all_reduce(view, group=self.group, async_op=True)
        elif self.mode == "zero":
            i = b.index
            o = self.shard_offsets[i]
            s, e = self.shard_ranges[i]
            if self.xdp is not None:
                ranges = [self.space.shard_range(b, r) for r in range(self.world)]
                b.work = self.xdp.reduce_scatter(self.space.grad_buf, ranges, self.grad_shard[o:o + (e - s)])
            else:
                b.work = comm.reduce_scatter_into(self.grad_shard[o:o + (e - s)], view, group=self.group, async_op=True)
        self._inflight.append(b)
        if self.overlap_optimizer:
            self._step_bucket_in_backward(b)

    def _step_bucket_in_backward(self, b):
        assert self._hparams is not None, "overlap_optimizer needs a FlatAdamW bound to this engine"
        lr, beta1, beta2, eps, wd = self._hparams()
        if not self._bwd_stepped:
            self._bwd_stepped = True
            self.step_count += 1
        if self.mode == "zero":
            self.wait_param_gather([b.index])  # last step's gather of this bucket (normally long done)
        scale = 1.0 / (self.grad_divisor * (self.accum_count + 1))  # this backward is micro-batch accum_count+1
        st = self._opt_stream
        if st is not None:
            st.wait_stream(torch.cuda.current_stream())  # this bucket's gradients are written
        with (torch.cuda.stream(st) if st is not None else contextlib.nullcontext()):
            if b.work is not None:
                b.work.wait()  # HIP: the side stream waits for the collective; gloo: blocks
            self._update_bucket(b, lr, beta1, beta2, eps, wd, scale)
            if self.mode == "zero":
                self._gather_bucket(b.index)
        b.stepped = True

    def _update_bucket(self, b, lr, beta1, beta2, eps, wd, scale):
        # `.data`: own version counter, so updating finished buckets in place does not trip
        # autograd's saved-tensor checks for weights later layers' backward still reads.
        buf = self.space.param_buf.data
        if self.mode == "zero":
            s, e = self.shard_ranges[b.index]
            o = self.shard_offsets[b.index]
            pv, gv, lo, hi = buf[s:e], self.grad_shard[o:o + (e - s)], o, o + (e - s)
        else:
            pv, gv, lo, hi = buf[b.start:b.end], self.space.grad_buf[b.start:b.end], b.start, b.end
        adamw_step(pv, gv, self.exp_avg[lo:hi], self.exp_avg_sq[lo:hi], lr=lr, step=self.step_count, beta1=beta1,
                   beta2=beta2, eps=eps, weight_decay=wd, grad_scale=scale,
                   master=None if self.master is None else self.master[lo:hi], hyper=self.graph_hyper)

    def finish_grad_sync(self):
        """Call after backward (the last micro-batch): flush unlaunched buckets, wait for all."""
        if self.mode == "single" and not self.overlap_optimizer and self._sync_enabled:
            self._reduce_sp()
        if (self.mode != "single" or self.overlap_optimizer) and self._sync_enabled:
            for p in self.params:
                if not getattr(p, "_dtg_grad_written", False):
                    p.main_grad.zero_()  # unused parameter this step
                    p._dtg_grad_written = True
            for b in self.space.buckets:
                if not b.launched:
                    self._launch(b)
            for b in self._inflight:
                if b.work is not None:
                    b.work.wait()
            self._inflight = []

    def backward(self, loss):
        loss.backward()
        self.accum_count += 1
        if self._sync_enabled:
            self.finish_grad_sync()

    def zero_grad(self):
        reset_grad_state(self.params)
        self._sp_reduced = False
        for b in self.space.buckets:
            b.pending = b.expected
            b.launched = False
            b.stepped = False
            b.work = None
        self.accum_count = 0

    # ------------------------------------------------------------------ optimizer
    def _shard_param_copy(self, out):
        if self.mode == "zero":
            for (s, e), o in zip(self.shard_ranges, self.shard_offsets):
                out[o:o + (e - s)].copy_(self.space.param_buf[s:e])
        else:
            out.copy_(self.space.param_buf)

    def step(self, lr, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.01, grad_scale=None):
        if self._bwd_stepped:  # overlap_optimizer: every bucket was updated during backward
            assert all(b.stepped for b in self.space.buckets), "a bucket missed its in-backward update"
            if self._opt_stream is not None:
                torch.cuda.current_stream().wait_stream(self._opt_stream)
            self._bwd_stepped = False
            return
        self.step_count += 1
        if grad_scale is None:
            grad_scale = 1.0 / (self.grad_divisor * max(1, self.accum_count))
        if self.mode == "zero":
            self.wait_param_gather()  # never update a slice an all-gather may still be reading
            if self._wt_stream is not None:  # ... or a W^T transpose
                torch.cuda.current_stream(self._wt_stream.device).wait_stream(self._wt_stream)
            for (s, e), o in zip(self.shard_ranges, self.shard_offsets):
                n = e - s
                adamw_step(self.space.param_buf[s:e], self.grad_shard[o:o + n], self.exp_avg[o:o + n],
                           self.exp_avg_sq[o:o + n], lr=lr, step=self.step_count, beta1=beta1, beta2=beta2,
                           eps=eps, weight_decay=weight_decay, grad_scale=grad_scale,
                           master=None if self.master is None else self.master[o:o + n], hyper=self.graph_hyper)
            if self._wt_buf is not None:
                self._wt_version = self.space.param_buf._version
                for b in self._wt_valid:
                    self._wt_valid[b] = False  # until the bucket's gather + transposes are issued
            self._allgather_params(wait=not self.overlap_param_gather)
        elif self._wt_buf is not None:  # same update + every weight's W^T for the next backward
            torch.ops.dtg.adamw_t_(self.space.param_buf, self.master, self.space.grad_buf, self.exp_avg,
                                   self.exp_avg_sq, self._wt_buf, self._wt_mats, int(self._wt_tiles), float(lr),
                                   float(beta1), float(beta2), float(eps), float(weight_decay), int(self.step_count),
                                   float(grad_scale), self.graph_hyper, self._wt_tc)
            self._wt_version = self.space.param_buf._version
        else:
            adamw_step(self.space.param_buf, self.space.grad_buf, self.exp_avg, self.exp_avg_sq, lr=lr,
                       step=self.step_count, beta1=beta1, beta2=beta2, eps=eps, weight_decay=weight_decay,
                       grad_scale=grad_scale, master=self.master, hyper=self.graph_hyper)

    def _allgather_params(self, wait: bool = True):
        """ZeRO: every rank updated its slice of each bucket; all-gather them in place, in the
        order the next forward needs them (`_ag_order`)."""
        gloo = comm.backend_of(self.group) == "gloo"
        order = getattr(self, "_ag_order", range(len(self.space.buckets)))
        # `.data` has its own version counter: the in-place gather (which may complete during the
        # next forward) must not invalidate weights autograd has already saved.
        for i in order:
            self._gather_bucket(i, gloo)
        if wait:
            self.wait_param_gather()

    def _gather_bucket(self, i, gloo=None):
        if gloo is None:
            gloo = comm.backend_of(self.group) == "gloo"
        buf = self.space.param_buf.data
        b = self.space.buckets[i]
        s, e = self.shard_ranges[i]
        src = buf[s:e]
        if self.xdp is not None:
            self._pending_ag[i] = self.xdp.all_gather(buf, [self.space.shard_range(b, r) for r in range(self.world)])
        else:
            self._pending_ag[i] = comm.all_gather_into(buf[b.start:b.end], src.clone() if gloo else src,
                                                       group=self.group, async_op=True)
        self._transpose_bucket(i, self._pending_ag[i])

    def wait_param_gather(self, buckets=None):
        for i in (list(self._pending_ag) if buckets is None else buckets):
            w = self._pending_ag.pop(i, None)
            if w is not None:
                w.wait()

    def _install_gather_hooks(self):
        """Map modules -> buckets they read: the root waits only for the embedding's buckets,
        each decoder layer for its own, and the final norm / untied lm_head buckets are waited
        for after the last layer.  Gathers are issued in that order, so the first layer starts
        as soon as the embedding has landed instead of behind the 1 GB lm_head gather."""
        bucket_of = {id(p): p._dtg_bucket.index for p in self.params}
        layers = list(getattr(self.module, "layers", []))
        in_layer = set()
        order = []
        for layer in layers:
            bs = sorted({bucket_of[id(p)] for p in layer.parameters() if id(p) in bucket_of})
            for p in layer.parameters():
                in_layer.add(id(p))
            layer.register_forward_pre_hook(lambda m, a, _bs=bs: self.wait_param_gather(_bs))
            order.extend(bs)
        outside = [p for p in self.params if id(p) not in in_layer]
        first = ("embed", "wte", "wpe")
        pre_bs = sorted({bucket_of[id(p)] for p in outside if any(k in getattr(p, "_dtg_name", "") for k in first)})
        post_bs = sorted({bucket_of[id(p)] for p in outside} - set(pre_bs))
        if not layers:
            pre_bs, post_bs = sorted(set(pre_bs) | set(post_bs)), []
        self.module.register_forward_pre_hook(lambda m, a: self.wait_param_gather(pre_bs))
        if post_bs:
            layers[-1].register_forward_hook(lambda m, a, o: self.wait_param_gather(post_bs))
        seen, ag_order = set(), []
        for i in pre_bs + order + post_bs + list(range(len(self.space.buckets))):
            if i not in seen:
                seen.add(i)
                ag_order.append(i)
        self._ag_order = ag_order

    def sync_params_after_load(self):
        if self.mode == "zero":
            self._allgather_params()

    # ------------------------------------------------------------------ checkpoint layout
    def ckpt_pieces(self):
        """This rank's owned slices: (param_name, start_in_param, numel, param_view, state_index).

        ddp/single own whole parameters (states indexed like the flat param buffer); zero owns
        the r-th slice of every bucket (states indexed in the shard space)."""
        self.wait_param_gather()
        sp = self.space
        out = []
        for i, name in enumerate(sp.names):
            off, n = sp.offsets[i], int(torch.Size(sp.shapes[i]).numel())
            if self.mode != "zero":
                out.append((name, 0, n, sp.param_buf[off:off + n], off))
                continue
            b = sp.param_bucket[i]
            s, e = self.shard_ranges[b.index]
            lo, hi = max(off, s), min(off + n, e)
            if lo < hi:
                out.append((name, lo - off, hi - lo, sp.param_buf[lo:hi], self.shard_offsets[b.index] + (lo - s)))
        return out

    def full_state_dict(self, rank0_only: bool = True):
        self.wait_param_gather()
        return {n: p.detach().cpu().clone() for n, p in self.module.named_parameters()}

    # ------------------------------------------------------------------ state
    def optimizer_state(self):
        st = {"step": self.step_count, "exp_avg": self.exp_avg, "exp_avg_sq": self.exp_avg_sq,
              "mode": self.mode, "world": self.world, "rank": self.rank}
        if self.master is not None:
            st["master"] = self.master
        return st

    def load_optimizer_state(self, st):
        assert st["mode"] == self.mode and st["world"] == self.world, "optimizer state layout mismatch"
        self.step_count = int(st["step"])
        self.exp_avg.copy_(st["exp_avg"])
        self.exp_avg_sq.copy_(st["exp_avg_sq"])
        if self.master is not None and "master" in st:
            self.master.copy_(st["master"])


class FlatAdamW(torch.optim.Optimizer):
    """torch.optim.Optimizer facade over an engine's fused flat AdamW (so schedulers work).

    Defaults follow torch.optim.AdamW as used by the reference (betas 0.9/0.999, eps 1e-8,
    weight_decay 0.01, pure-bf16 states)."""

    def __init__(self, engine, lr=3e-5, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.01):
        self.engine = engine
        params = [p for p in engine.module.parameters() if p.requires_grad]
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        if hasattr(engine, "_hparams"):
            g = self.param_groups[0]
            engine._hparams = lambda: (g["lr"], g["betas"][0], g["betas"][1], g["eps"], g["weight_decay"])

    @torch.no_grad()
    def step(self, closure=None):
        g = self.param_groups[0]
        self.engine.step(g["lr"], g["betas"][0], g["betas"][1], g["eps"], g["weight_decay"])

    def zero_grad(self, set_to_none: bool = True):
        self.engine.zero_grad()

    def state_dict(self):
        return {"param_groups": [{k: v for k, v in g.items() if k != "params"} for g in self.param_groups],
                "engine": self.engine.optimizer_state()}

    def load_state_dict(self, sd):
        for g, sg in zip(self.param_groups, sd["param_groups"]):
            g.update(sg)
        self.engine.load_optimizer_state(sd["engine"])
