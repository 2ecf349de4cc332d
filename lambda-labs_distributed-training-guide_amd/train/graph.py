"""HIP-graph capture of a whole training step (forward + backward + AdamW) for launch-bound
configurations.

A step of this framework is a few hundred to a few thousand kernel launches.  For the big
models every launch is long and the host runs far ahead, but for small ones (GPT-2 124M, the
chapter 01/02 default, short sequences, small batches) the step is bounded by launch latency.
`GraphedStep` records the step once into a HIP graph (`torch.cuda.CUDAGraph` is hipGraph on
ROCm) and replays it with one launch per step -- the MI355X-native replacement for a tracing
compiler's "reduce overhead" mode.

What makes a step replayable:
  * inputs are copied into static device buffers before each replay;
  * the optimizer's step-dependent scalars (learning rate, bias corrections) are read by the
    AdamW kernel from a device tensor the host rewrites before each replay
    (`DataParallel.graph_hyper`); the LR scheduler keeps running on the host;
  * the loss stays on the device (`.item()` only when the caller logs);
  * gradient routing flags are reset by the captured `zero_grad`, so the captured kernel
    sequence (first gradient contribution writes, later ones accumulate) is valid every step.

Single-process engines only (`DataParallel` mode "single"); collectives are not captured.
Create the GraphedStep before running any eager step of the model (see `_stream`).
"""
from __future__ import annotations

import math
from typing import Dict, Optional

import torch


class GraphedStep:
    def __init__(self, model, engine, optimizer, scheduler=None, warmup: int = 3, num_valid: Optional[int] = None):
        assert getattr(engine, "mode", None) == "single", "GraphedStep captures single-process engines only"
        assert not getattr(engine, "overlap_optimizer", False), "capture the plain post-backward optimizer step"
        self.model, self.engine, self.opt, self.sched = model, engine, optimizer, scheduler
        self.warmup = warmup
        self.num_valid = num_valid
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self.static: Dict[str, torch.Tensor] = {}
        self.loss: Optional[torch.Tensor] = None
        dev = next(model.parameters()).device
        # pinned staging ring: the host fills slot i only after slot i's previous H2D copy ran
        self._ring = [torch.zeros(3, dtype=torch.float32, pin_memory=True) for _ in range(4)]
        self._ring_ev = [None] * len(self._ring)
        self._slot = 0
        self._hyper = torch.zeros(3, dtype=torch.float32, device=dev)
        # One side stream for the eager warm-up steps AND the capture: autograd's AccumulateGrad
        # nodes (ATen-gradient parameters such as GPT-2's LayerNorm) bind to the stream they
        # were created on, and must match the capturing stream.
        self._stream = torch.cuda.Stream(device=dev)
        self.steps = 0

    # ------------------------------------------------------------------ eager step
    def _eager(self, batch):
        self.opt.zero_grad()
        out = self.model(**batch, num_valid=self.num_valid) if self.num_valid is not None else self.model(**batch)
        self.engine.backward(out.loss)
        self.opt.step()
        return out.loss

    def _write_hyper(self):
        """Values for the step the next replay performs (engine.step_count + 1)."""
        g = self.opt.param_groups[0]
        t = self.engine.step_count + 1
        b1, b2 = g["betas"]
        i = self._slot
        self._slot = (i + 1) % len(self._ring)
        if self._ring_ev[i] is not None:
            self._ring_ev[i].synchronize()
        host = self._ring[i]
        host[0] = g["lr"]
        host[1] = 1.0 - b1 ** t
        host[2] = math.sqrt(1.0 - b2 ** t)
        self._hyper.copy_(host, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self._ring_ev[i] = ev

    def _capture(self, batch):
        """Record one step (nothing executes during capture; the first replay performs it)."""
        self.static = {k: v.clone() for k, v in batch.items()}
        self.engine.graph_hyper = self._hyper
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        count = self.engine.step_count
        with torch.cuda.graph(self.graph, stream=self._stream):
            self.loss = self._eager(self.static)
        self.engine.step_count = count  # capture ran the host code once: roll its counter back

    # ------------------------------------------------------------------ step
    def _replayable(self, batch, num_valid) -> bool:
        if num_valid is not None and num_valid != self.num_valid:
            return False
        return (set(batch) == set(self.static) and
                all(v.shape == self.static[k].shape and v.dtype == self.static[k].dtype for k, v in batch.items()))

    def __call__(self, batch, num_valid: Optional[int] = None) -> torch.Tensor:
        """One training step on `batch`; returns the device loss.

        The first `warmup` calls run eagerly on a side stream (lazy initialisation, allocator
        warm-up, as graph capture requires); the next call captures the step and every call
        from then on replays it.  A batch that does not fit the captured one (other shapes or
        keys, or another `num_valid` -- the loss scale is part of the graph) runs eagerly on
        the same stream.  Training semantics are those of the eager loop."""
        if num_valid is not None and self.num_valid is None:
            self.num_valid = num_valid
        eager = self.graph is None and self.steps < self.warmup
        if self.graph is not None and not self._replayable(batch, num_valid):
            eager = True
        if eager:
            s = self._stream
            s.wait_stream(torch.cuda.current_stream())
            saved_nv = self.num_valid
            if num_valid is not None:
                self.num_valid = num_valid
            with torch.cuda.stream(s):
                if self.graph is not None:
                    self._write_hyper()  # the engine reads AdamW scalars from the device now
                loss = self._eager(batch)
            self.num_valid = saved_nv
            torch.cuda.current_stream().wait_stream(s)
        else:
            if self.graph is None:
                self._capture(batch)
            # replay on the capture stream, ordered after the caller's stream both ways
            s = self._stream
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                for k, v in batch.items():
                    self.static[k].copy_(v, non_blocking=True)
                self._write_hyper()
                self.graph.replay()
            torch.cuda.current_stream().wait_stream(s)
            for v in batch.values():
                v.record_stream(s)
            self.engine.step_count += 1
            loss = self.loss
        if self.sched is not None:
            self.sched.step()
        self.steps += 1
        return loss
