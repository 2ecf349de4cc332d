"""Pipeline parallelism: Llama decoder layers split into stages, one-forward-one-backward
(1F1B) micro-batch schedule, activations exchanged point to point (SURVEY §2.3 "PP" stretch
row; the reference only names "pipeline/model parallel" in 06-tensor-parallel/README.md).

Why it is shaped this way on MI355X:
  * A stage boundary moves one [2, tokens, hidden] bf16 tensor (the residual stream and the
    last sub-block output, whose add is fused into the next RMSNorm) per micro-batch in each
    direction -- 64 MiB for 8 x 1024 tokens at hidden 4096, ~0.5 ms over one xGMI link.
    Every GPU pair of a node has its own link, so the P-1 boundaries of a pipeline never share
    a link and run concurrently.
  * The 1F1B order bounds live activations at (P - stage) micro-batches per stage.  Sends and
    receives that cross in time are issued as one batch_isend_irecv (send-forward+recv-backward
    / send-backward+recv-forward pairs), the pattern RCCL executes without deadlock.
  * 288 GB of HBM per GPU means pipeline depth is a choice for very deep models (405B at 126
    layers) or few-GPU nodes, not a necessity; it composes with data parallel replicas of each
    stage (`DataParallel` over the stage's dp group).

Stage layout: stage 0 owns the embedding, the last stage the final norm and the loss head (and
the embedding too when it is tied to the lm_head; the two copies' gradients are summed over a
first/last group before the data-parallel sync).  `balanced_partition` gives the last stage
fewer layers to offset the vocabulary GEMM.
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import torch
import torch.distributed as dist
import torch.nn as nn

from ..utils import comm


def balanced_partition(num_layers: int, stages: int, head_cost_layers: float = 0.0) -> List[int]:
    """Layers per stage, with the last stage charged `head_cost_layers` extra (its loss head).

    Llama-3-8B: the 128k-vocabulary head is ~2.4 decoder layers of FLOPs (2*H*V vs 2*H*(qkv+o+3I))."""
    assert num_layers >= stages, f"{num_layers} layers cannot fill {stages} stages"
    total = num_layers + head_cost_layers
    per = total / stages
    sizes, done = [], 0
    for s in range(stages):
        left = stages - s - 1
        if left == 0:
            n = num_layers - done
        else:
            n = int(round(per * (s + 1))) - done
            n = max(1, min(n, num_layers - done - left))
        sizes.append(n)
        done += n
    return sizes


def head_cost_in_layers(cfg) -> float:
    h, i, v = cfg.hidden_size, cfg.intermediate_size, cfg.vocab_size
    d = cfg.head_dim
    layer = h * (cfg.num_attention_heads * d * 2 + cfg.num_key_value_heads * d * 2) + 3 * h * i
    return h * v / layer


def _global_rank(group, r: int) -> int:
    return r if group is None else dist.get_global_rank(group, r)


class PipelineStage:
    """Prune a LlamaForCausalLM in place down to this rank's stage of a `group` pipeline."""

    def __init__(self, model: nn.Module, group=None, partition: Optional[Sequence[int]] = None,
                 balanced: bool = True):
        assert getattr(model, "tp", None) is None or not model.tp.enabled, "PP is not combined with TP here"
        assert model.cp_group is None and model.sp_group is None, "PP is not combined with CP / Ulysses here"
        self.model = model
        self.group = group
        self.size = comm.world(group) if dist.is_initialized() else 1
        self.stage = comm.rank(group) if self.size > 1 else 0
        n = len(model.layers)
        if partition is None:
            partition = balanced_partition(n, self.size, head_cost_in_layers(model.config) if balanced else 0.0)
        assert len(partition) == self.size and sum(partition) == n and min(partition) >= 1, partition
        self.partition = list(partition)
        a = sum(partition[:self.stage])
        self.layer_range = (a, a + partition[self.stage])
        self.first, self.last = self.stage == 0, self.stage == self.size - 1
        model.layers = nn.ModuleList(list(model.layers)[a:a + partition[self.stage]])
        self.tied = model.lm_head is None
        if not self.first and not (self.last and self.tied):
            model.embed_tokens = None
        if not self.last:
            model.norm = None
            model.lm_head = None
        self.tie_group = None
        if self.size > 1 and self.tied and model.embed_tokens is not None:
            model.embed_tokens.weight._dtg_uses = 1  # one use per stage (embedding, or lm_head)
            if not self.first:  # the last stage's copy of the tied matrix: checkpointed by stage 0
                model._dtg_ckpt_skip = {"embed_tokens.weight"}
        if self.size > 1 and self.tied:
            # first + last stage of every pipeline (new_group is collective over the world)
            W, P = dist.get_world_size(), self.size
            me = dist.get_rank()
            for start in range(0, W, P):
                g = dist.new_group([start, start + P - 1])
                if start <= me < start + P:
                    self.tie_group = g if (self.first or self.last) else None
        self.prev = _global_rank(group, self.stage - 1) if (self.size > 1 and not self.first) else None
        self.next = _global_rank(group, self.stage + 1) if (self.size > 1 and not self.last) else None


class OneFOneB:
    """1F1B schedule over `num_microbatches` equal row splits of each batch.

    step() runs forward + backward of the whole batch and leaves the stage's gradients in the
    engine (`DataParallel` over this stage's dp group, or mode="single"); the caller then runs the
    optimizer.  Returns the batch loss (the mean over all valid labels) on every stage."""

    def __init__(self, stage: PipelineStage, engine, num_microbatches: int):
        self.st = stage
        self.engine = engine
        self.m = num_microbatches
        self.model = stage.model
        self._gloo = stage.size > 1 and comm.backend_of(stage.group) == "gloo"

    # -------------------------------------------------------------- point to point
    def _p2p(self, send=None, send_to=None, recv_like=None, recv_from=None):
        # gloo moves host memory only: device tensors are staged through the host there (the
        # 1-GPU rehearsals); RCCL sends device buffers directly over xGMI
        host = self._gloo and (recv_like if recv_like is not None else send).is_cuda
        ops, out = [], None
        if send is not None:
            ops.append(dist.P2POp(dist.isend, send.cpu() if host else send.contiguous(), send_to, self.st.group))
        if recv_like is not None:
            out = torch.empty(recv_like.shape, dtype=recv_like.dtype, device="cpu" if host else recv_like.device)
            ops.append(dist.P2POp(dist.irecv, out, recv_from, self.st.group))
        if ops:
            for w in dist.batch_isend_irecv(ops):
                w.wait()
        if host and out is not None:
            out = out.to(recv_like.device)
        return out

    # -------------------------------------------------------------- compute
    def _forward(self, i, inp):
        mb = self.mbs[i]
        rc = self.model.run_context(mb["input_ids"], mb.get("position_ids"))
        if self.st.first:
            x, res = self.model.embed(mb["input_ids"]), None
        else:
            x, res = inp[0], inp[1]
        for layer in self.model.layers:
            x, res = layer(x, res, rc)
        if self.st.last:
            out = self.model.head(x, res, mb["labels"], num_valid=self.num_valid)
            return out.loss
        return torch.stack([x, res])

    def step(self, input_ids, labels=None, num_valid=None, position_ids=None):
        st, m, model = self.st, self.m, self.model
        B = input_ids.shape[0]
        assert B % m == 0, f"batch {B} must split into {m} micro-batches"
        labels = input_ids if labels is None else labels
        if num_valid is None:
            num_valid = int((labels[:, 1:] != -100).sum())
        self.num_valid = num_valid
        rows = B // m
        self.mbs = [{"input_ids": input_ids[j * rows:(j + 1) * rows], "labels": labels[j * rows:(j + 1) * rows],
                     **({} if position_ids is None else {"position_ids": position_ids[j * rows:(j + 1) * rows]})}
                    for j in range(m)]
        if hasattr(self.engine, "wait_param_gather"):
            self.engine.wait_param_gather()  # ZeRO gathers wait in the root forward hook, not called here
        H = model.config.hidden_size
        dt = next(p for p in model.parameters()).dtype
        act_like = torch.empty(2, rows * input_ids.shape[1], H, dtype=dt, device=input_ids.device)
        warm = min(st.size - st.stage - 1, m)
        inputs, outputs = [None] * m, [None] * m
        loss_sum = torch.zeros((), dtype=torch.float32, device=input_ids.device)
        fwd_i = bwd_i = 0
        recv = None if st.first else self._p2p(recv_like=act_like, recv_from=st.prev)

        def run_fwd():
            nonlocal fwd_i, recv
            inp = None
            if not st.first:
                inp = recv.requires_grad_()
            out = self._forward(fwd_i, inp)
            inputs[fwd_i], outputs[fwd_i] = inp, out
            fwd_i += 1
            return out

        def run_bwd(grad):
            nonlocal bwd_i
            out = outputs[bwd_i]
            with self.engine.no_sync():
                if st.last:
                    out.backward()
                else:
                    torch.autograd.backward(out, grad)
            gin = None if st.first else inputs[bwd_i].grad
            inputs[bwd_i] = outputs[bwd_i] = None
            bwd_i += 1
            return gin

        # warmup: forwards only
        for _ in range(warm):
            out = run_fwd()
            nxt = fwd_i < m and not st.first
            self._p2p(send=out.detach(), send_to=st.next)
            recv = self._p2p(recv_like=act_like, recv_from=st.prev) if nxt else None
        # steady state: one forward, one backward
        for k in range(m - warm):
            out = run_fwd()
            if st.last:
                loss_sum += out.detach().float()
                grad = None
            else:  # send this activation, receive the gradient of the oldest in-flight one
                grad = self._p2p(send=out.detach(), send_to=st.next, recv_like=act_like, recv_from=st.next)
            gin = run_bwd(grad)
            last_steady = k == m - warm - 1
            if st.first:
                continue
            if last_steady:
                self._p2p(send=gin, send_to=st.prev)
            else:  # send the input gradient, receive the next forward's input
                recv = self._p2p(send=gin, send_to=st.prev, recv_like=act_like, recv_from=st.prev)
        # cooldown: backwards only
        for _ in range(warm):
            grad = self._p2p(recv_like=act_like, recv_from=st.next)
            gin = run_bwd(grad)
            if not st.first:
                self._p2p(send=gin, send_to=st.prev)
        self._finish(loss_sum)
        return self.loss

    def _finish(self, loss_sum):
        st = self.st
        if st.tie_group is not None:  # embedding (stage 0) and lm_head (last stage) are one matrix
            g = self.model.embed_tokens.weight.main_grad
            dist.all_reduce(g, group=st.tie_group)
        eng = self.engine
        if hasattr(eng, "finish_grad_sync"):
            eng.finish_grad_sync()  # data-parallel replicas of this stage
        # every stage reports the batch loss (it lives on the last stage)
        if st.size > 1:
            src = _global_rank(st.group, st.size - 1)
            dist.broadcast(loss_sum, src=src, group=st.group)
        self.loss = loss_sum
