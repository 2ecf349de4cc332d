"""Llama-family causal LM (Llama-2/3/3.1/3.2, GQA, llama3 RoPE scaling, tied embeddings).

Owned by this repo instead of HF transformers so the layout fits the kernels:
  * fused QKV weight [(nq + 2 nkv) * d, H] and fused gate|up weight [2 I, H] (one hipBLASLt
    GEMM each; attention reads q/k/v straight out of the fused output);
  * the residual add is fused into the following RMSNorm (`add_rms_norm`);
  * RoPE is applied inside the attention autograd node (in place on the QKV activation);
  * lm_head + cross entropy are fused and chunked (no [T, V] logits in memory);
  * activations are 2-D token-major [B*S, H]; packed sequences (position ids restarting at
    EOS, 00-rime) go through varlen attention via cu_seqlens.
Tensor parallelism (Megatron column/row + sequence parallel + vocab-parallel embedding and
loss) is built in: pass `tp_group` and every weight is the local shard.

State-dict names follow HF (`model.layers.N.self_attn.qkv_proj.weight`, ...); `hf_compat`
converts to/from HF's split q/k/v and gate/up tensors.
"""
from __future__ import annotations

import dataclasses
import weakref
from typing import Optional

import torch
import torch.distributed as dist
import torch.nn as nn

from .. import ops
from ..parallel import async_tp, tp_comm
from .config import LlamaConfig


@dataclasses.dataclass
class CausalLMOutput:
    loss: Optional[torch.Tensor] = None
    logits: Optional[torch.Tensor] = None


class Weight(nn.Module):
    """Parameter holder (no forward); keeps HF-like `<name>.weight` state-dict keys."""

    _dtg_param_holder = True

    def __init__(self, *shape, device=None, dtype=torch.bfloat16):
        super().__init__()
        self.weight = nn.Parameter(torch.empty(*shape, device=device, dtype=dtype))


class TPInfo:
    def __init__(self, group=None):
        self.group = group
        self.size = dist.get_world_size(group) if group is not None else 1
        self.rank = dist.get_rank(group) if group is not None else 0
        # chunks of the overlapped sequence-parallel regions (parallel/async_tp.py; 1 = the
        # synchronous gather -> block -> scatter path)
        self.overlap_chunks = async_tp.DEFAULT_CHUNKS
        # re-gather the sequence-parallel inputs in the backward instead of keeping them
        # (`--sp-regather`, parallel/async_tp.py `regathered`; layers that recompute skip it)
        self.sp_regather = False

    @property
    def enabled(self):
        return self.size > 1


class RunCtx:
    """Per-forward runtime data shared by all layers."""

    __slots__ = ("cos", "sin", "pos", "cu_seqlens", "max_seqlen", "cp_group", "rows", "sp_group", "cp_ranges")

    def __init__(self, cos, sin, pos, cu_seqlens, max_seqlen, cp_group=None, rows=0, sp_group=None, cp_ranges=None):
        self.cos, self.sin, self.pos, self.cu_seqlens, self.max_seqlen = cos, sin, pos, cu_seqlens, max_seqlen
        self.cp_group, self.rows, self.sp_group = cp_group, rows, sp_group
        self.cp_ranges = cp_ranges  # context parallel over packed rows (parallel/context_parallel.py)


class LlamaAttention(nn.Module):
    def __init__(self, cfg: LlamaConfig, tp: TPInfo, device=None, dtype=torch.bfloat16):
        super().__init__()
        assert cfg.num_attention_heads % tp.size == 0 and cfg.num_key_value_heads % tp.size == 0, \
            "tensor-parallel degree must divide the number of query and key/value heads"
        self.nq = cfg.num_attention_heads // tp.size
        self.nkv = cfg.num_key_value_heads // tp.size
        self.d = cfg.head_dim
        h = cfg.hidden_size
        self.qkv_proj = Weight((self.nq + 2 * self.nkv) * self.d, h, device=device, dtype=dtype)
        if cfg.attention_bias:  # Qwen2: q/k/v biases, fused like the weight; a [rows, 1] column so
            # that tensor-parallel sharding and checkpoint geometry treat it like the weight's rows
            self.qkv_proj.bias = nn.Parameter(torch.empty((self.nq + 2 * self.nkv) * self.d, 1, device=device,
                                                          dtype=dtype))
        self.o_proj = Weight(h, self.nq * self.d, device=device, dtype=dtype)
        self.window = int(cfg.sliding_window or 0)

    def forward(self, x, rc: RunCtx, out=None):
        b = getattr(self.qkv_proj, "bias", None)
        qkv = ops.linear(x, self.qkv_proj.weight, None if b is None else b.view(-1))
        if rc.cp_group is not None:  # context parallel: zig-zag sequence shards
            from ..parallel.context_parallel import cp_attention

            T, d = qkv.shape[0], self.d
            qkv = ops.rope(qkv, rc.cos, rc.sin, rc.pos, self.nq + self.nkv, d)
            q = qkv[:, :self.nq * d].reshape(T, self.nq, d)
            k = qkv[:, self.nq * d:(self.nq + self.nkv) * d].reshape(T, self.nkv, d)
            v = qkv[:, (self.nq + self.nkv) * d:].reshape(T, self.nkv, d)
            o = cp_attention(q, k, v, rc.cp_group, rc.rows, ranges=rc.cp_ranges).reshape(T, self.nq * d)
        elif rc.sp_group is not None:  # Ulysses: all-to-all to full sequences x local heads
            from ..parallel.ulysses import ulysses_attention

            o = ulysses_attention(qkv, self.nq, self.nkv, self.d, rc.sp_group, rc.rows, rc.cu_seqlens,
                                  rc.max_seqlen, rc.cos, rc.sin, rc.pos)
        else:
            o = ops.attention(qkv, self.nq, self.nkv, self.d, rc.cu_seqlens, rc.max_seqlen, rc.cos, rc.sin, rc.pos,
                              window=self.window)
        return ops.linear(o, self.o_proj.weight, out=out)


class LlamaMLP(nn.Module):
    def __init__(self, cfg: LlamaConfig, tp: TPInfo, device=None, dtype=torch.bfloat16):
        super().__init__()
        assert cfg.intermediate_size % tp.size == 0
        self.inter = cfg.intermediate_size // tp.size
        self.gate_up_proj = Weight(2 * self.inter, cfg.hidden_size, device=device, dtype=dtype)
        self.down_proj = Weight(cfg.hidden_size, self.inter, device=device, dtype=dtype)

    def forward(self, x, out=None):
        return ops.swiglu_mlp(x, self.gate_up_proj.weight, self.down_proj.weight, out=out)


class LlamaDecoderLayer(nn.Module):
    def __init__(self, cfg: LlamaConfig, tp: TPInfo, device=None, dtype=torch.bfloat16):
        super().__init__()
        self.eps = cfg.rms_norm_eps
        self.tp = tp
        self.input_layernorm = Weight(cfg.hidden_size, device=device, dtype=dtype)
        self.post_attention_layernorm = Weight(cfg.hidden_size, device=device, dtype=dtype)
        self.self_attn = LlamaAttention(cfg, tp, device, dtype)
        self.mlp = LlamaMLP(cfg, tp, device, dtype)
        for p in (self.input_layernorm.weight, self.post_attention_layernorm.weight):
            p._dtg_sequence_parallel = tp.enabled  # replicated over TP; grads need a TP all-reduce

    def forward(self, x, res, rc: RunCtx):
        """x: previous sub-block output (or embeddings), res: residual stream (None at layer 0).
        Returns (mlp output, residual stream); the residual add is fused into the next norm."""
        g = self.tp.group if self.tp.enabled else None
        if res is None:
            n, res = ops.rms_norm(x, self.input_layernorm.weight, self.eps), x
        else:
            n, res = ops.add_rms_norm(x, res, self.input_layernorm.weight, self.eps)
        ka, km = self._overlap_chunks(n.shape[0], rc) if g is not None else (1, 1)
        regather = g is not None and self._regather()
        if ka > 1:
            a = async_tp.sp_region(n, lambda xg, j, out=None: self.self_attn(xg, _chunk_ctx(rc, xg.shape[0]), out=out), g, ka,
                                   tuple(p for p in self.self_attn.parameters()), regather=regather)
        elif g is not None:
            a = self._sp_block(n, lambda xg: self.self_attn(xg, rc), g, regather)
        else:
            a = self.self_attn(n, rc)
        n2, res = ops.add_rms_norm(a, res, self.post_attention_layernorm.weight, self.eps)
        if km > 1:
            m = async_tp.sp_region(n2, lambda xg, j, out=None: self.mlp(xg, out=out), g, km,
                                   (self.mlp.gate_up_proj.weight, self.mlp.down_proj.weight), regather=regather)
        elif g is not None:
            m = self._sp_block(n2, self.mlp, g, regather)
        else:
            m = self.mlp(n2)
        return m, res

    def _regather(self):
        return self.tp.sp_regather and torch.is_grad_enabled() and not getattr(self, "_dtg_checkpointed", False)

    @staticmethod
    def _sp_block(n, fn, g, regather):
        """Synchronous sequence-parallel sub-block: gather -> fn -> reduce-scatter.  With regather
        the gathered input is not kept for fn's backward (async_tp.regathered): it is re-gathered,
        the all-gather issued as soon as the sub-block's output gradient arrives."""
        full = tp_comm.gather_seq(n, g)
        if not regather:
            return tp_comm.scatter_seq(fn(full), g)
        with async_tp.regathered(full, n, g) as h:
            y = fn(full)
        if y.requires_grad:
            # weak: the hook lives on in the graph until the step's output is released; the
            # handle (and the rows it holds) must not
            ref = weakref.ref(h)
            y.register_hook(lambda grad: None if ref() is None else ref().prefetch())
        return tp_comm.scatter_seq(y, g)

    def _overlap_chunks(self, rows_local, rc: RunCtx):
        """(attention, MLP) chunk counts of the overlapped SP regions for this forward."""
        k = self.tp.overlap_chunks
        if k <= 1 or getattr(self, "_dtg_checkpointed", False) or not torch.is_grad_enabled():
            return 1, 1
        km = async_tp.region_chunks(rows_local, k)
        dense = (rc.cp_group is None and rc.sp_group is None and rc.cu_seqlens is not None
                 and rc.cu_seqlens.numel() == rc.rows + 1 and rc.max_seqlen > 0)
        ka = async_tp.region_chunks(rows_local, k, rc.max_seqlen) if dense else 1
        return ka, km


def tp_seed_offset(tp_rank: int) -> int:
    """Seed offset of TP rank `tp_rank`'s sharded-weight initialisation (0 for rank 0)."""
    return 1_000_003 * int(tp_rank)


def _chunk_ctx(rc: RunCtx, rows: int) -> RunCtx:
    """RunCtx of a gathered chunk of whole dense rows (`rows` tokens = rows // S sequences)."""
    S = rc.max_seqlen
    b = rows // S
    return RunCtx(rc.cos, rc.sin, rc.pos[:rows], rc.cu_seqlens[:b + 1], S, None, b, None)


class _VocabParallelEmbedding(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, w, vstart):
        from ..utils.comm import _FAKE

        local = ids - vstart
        if _FAKE:
            # DTG_FAKE_WORLD rehearsal: the other ranks' rows of this sum never arrive, so a token
            # outside this shard would keep an all-zero hidden state -- for the first token of a
            # sequence through every layer (it attends only to itself), and each RMSNorm backward
            # then multiplies its gradient by 1/sqrt(eps) until bf16 overflows
            # (profiles/r5/fake_nan/).  Every token takes a row of this shard instead (same cost).
            local = torch.remainder(local, w.shape[0])
        mask = (local < 0) | (local >= w.shape[0])
        local = local.masked_fill(mask, 0)
        out = torch.nn.functional.embedding(local, w)
        out.masked_fill_(mask[:, None], 0)
        ctx.save_for_backward(local, mask)
        ctx.w = w
        return out

    @staticmethod
    def backward(ctx, dy):
        local, mask = ctx.saved_tensors
        from ..ops.grad_routing import route_embedding_grad

        # out-of-shard tokens get id -1, which embedding_bwd_ skips: no zeroed dy copy, and no
        # single run of ~(tp-1)/tp of all tokens on row 0 for the segment sum to walk
        return None, route_embedding_grad(ctx.w, local.masked_fill(mask, -1), dy.contiguous(), ctx.w.shape[0]), None


class LlamaForCausalLM(nn.Module):
    def __init__(self, cfg: LlamaConfig, tp_group=None, device=None, dtype=torch.bfloat16, cp_group=None,
                 sp_group=None):
        super().__init__()
        self.config = cfg
        self.tp = TPInfo(tp_group)
        # context parallel (parallel/context_parallel.py): inputs are zig-zag sequence shards with
        # global position_ids and labels already shifted on the full sequence (cp_batch)
        self.cp_group = cp_group
        # Ulysses sequence parallel (parallel/ulysses.py): inputs are contiguous sequence slices,
        # labels shifted on the full rows (ulysses_batch), position_ids (packed rows) local slices
        self.sp_group = sp_group
        assert sum(g is not None for g in (cp_group, tp_group, sp_group)) <= 1, \
            "context, Ulysses and tensor parallelism are not combined"
        tp = self.tp
        assert cfg.vocab_size % tp.size == 0 or not tp.enabled, "vocab must divide by the TP degree"
        self.vocab_local = cfg.vocab_size // tp.size
        self.vocab_start = tp.rank * self.vocab_local
        self.embed_tokens = Weight(self.vocab_local, cfg.hidden_size, device=device, dtype=dtype)
        self.layers = nn.ModuleList([LlamaDecoderLayer(cfg, tp, device, dtype) for _ in range(cfg.num_hidden_layers)])
        self.norm = Weight(cfg.hidden_size, device=device, dtype=dtype)
        self.norm.weight._dtg_sequence_parallel = tp.enabled
        self.lm_head = None if cfg.tie_word_embeddings else Weight(self.vocab_local, cfg.hidden_size, device=device, dtype=dtype)
        if cfg.tie_word_embeddings:
            self.embed_tokens.weight._dtg_uses = 2  # embedding + lm_head gradient contributions
        self._rope = None
        self._dense_cache = {}

    # ---------------------------------------------------------------- init
    @torch.no_grad()
    def init_param(self, name: str, t: torch.Tensor):
        """HF Llama init: normal(0, initializer_range) for matrices/embeddings, ones for norms."""
        if name.endswith("layernorm.weight") or name == "norm.weight":
            t.fill_(1.0)
        elif name.endswith(".bias"):
            t.zero_()
        else:
            t.normal_(0.0, self.config.initializer_range)

    @torch.no_grad()
    def init_weights(self):
        """Under TP every rank holds a different slice of each sharded matrix, so every rank must
        draw different values: the ranks of a TP group share the global RNG seed (same data order,
        same replicated norms), and the sharded weights are drawn with that seed offset by the TP
        rank (`tp_seed_offset`).  With identical draws the column / row blocks of all TP ranks
        would be copies of each other, receive identical gradients and never diverge."""
        off = tp_seed_offset(self.tp.rank) if self.tp.enabled else 0
        for name, p in self.named_parameters():
            if p.device.type == "meta":
                continue
            if off:
                state = torch.random.get_rng_state()
                torch.manual_seed((int(torch.randint(0, 2**62, (1,)).item()) + off) % 2**63)
                self.init_param(name, p)
                torch.random.set_rng_state(state)
                torch.randint(0, 2**62, (1,))  # advance the shared stream identically on all ranks
            else:
                self.init_param(name, p)

    def lm_head_weight(self):
        return self.embed_tokens.weight if self.lm_head is None else self.lm_head.weight

    # ---------------------------------------------------------------- runtime
    def _rope_tables(self, need: int, device):
        if self._rope is None or self._rope[0].shape[0] < need or self._rope[0].device != device:
            n = max(need, 4096)
            n = (n + 4095) // 4096 * 4096
            c = self.config
            self._rope = ops.rope_tables(c.head_dim, c.rope_theta, n, c.rope_scaling, device=device)
        return self._rope

    def _dense_meta(self, B, S, device):
        key = (B, S, str(device))
        v = self._dense_cache.get(key)
        if v is None:
            pos = torch.arange(S, device=device, dtype=torch.long).repeat(B)
            cu = torch.arange(0, (B + 1) * S, S, device=device, dtype=torch.int32)
            v = (pos, cu)
            self._dense_cache = {key: v}
        return v

    def forward(self, input_ids, labels=None, position_ids=None, cu_seqlens=None, max_seqlen=None,
                num_valid=None, return_logits=False, attention_mask=None):
        """HF-compatible call: model(input_ids=[B,S], labels=[B,S], position_ids=[B,S]?).

        Packed sequences: pass position_ids (restarting at 0 per document) and ideally
        cu_seqlens (int32 [ndocs+1]) + max_seqlen from the collator (else derived, 1 sync).
        `num_valid` (host int) = number of non-ignored shifted labels (avoids a sync)."""
        rc = self.run_context(input_ids, position_ids, cu_seqlens, max_seqlen)
        x, res = self.embed(input_ids), None
        for layer in self.layers:
            x, res = layer(x, res, rc)
        return self.head(x, res, labels, num_valid, return_logits, input_ids.shape[0])

    # The three pieces of forward, also driven one by one by the pipeline-parallel stages
    # (parallel/pipeline.py): run_context -> embed -> layers -> head.
    def run_context(self, input_ids, position_ids=None, cu_seqlens=None, max_seqlen=None) -> RunCtx:
        """Per-forward attention metadata (positions, varlen boundaries, RoPE tables)."""
        B, S = input_ids.shape
        T = B * S
        dev = input_ids.device
        sw = self.config.sliding_window
        if sw is not None and (self.cp_group is not None or self.sp_group is not None) and S > sw:
            raise ValueError(f"{self.config.model_type}: context / Ulysses parallelism with rows longer than the "
                             f"sliding window ({sw}) is not supported; the single-rank and TP paths are")
        sp = self.sp_group is not None
        if sp:  # attention sees the full rows: describe them (positions gathered from the slices)
            from ..parallel.ulysses import sp_world

            n = sp_world(self.sp_group)
            if position_ids is not None:
                from ..utils import comm

                loc = position_ids.to(device=dev, dtype=torch.long).contiguous()
                position_ids = comm.all_gather_dim0(loc.t().contiguous(), self.sp_group).t()  # [B, n*S]
                cu_seqlens = None
            S = S * n
            T = B * S
        cp_ranges = None
        if self.cp_group is not None:  # attention over zig-zag chunks; cu_seqlens (if given) are the
            # FULL rows' document boundaries of a packed batch (cp_batch keeps the collator's)
            if cu_seqlens is not None:  # built on the device: no host sync per forward
                from ..parallel.context_parallel import cp_ranges as _cp_ranges
                from ..utils import comm

                n = comm.world(self.cp_group)
                cp_ranges = _cp_ranges(comm.rank(self.cp_group), n, B, S // 2, dev, cu_seqlens=cu_seqlens)
            pos, cu, max_seqlen = position_ids.reshape(-1).to(torch.long), None, 0
        elif position_ids is None:
            pos, cu = self._dense_meta(B, S, dev)
            max_seqlen = S
        else:
            pos = position_ids.reshape(-1).to(torch.long)
            if cu_seqlens is None:
                starts = torch.nonzero(pos == 0).flatten()
                row_starts = torch.arange(0, T, S, device=dev)
                starts = torch.unique(torch.cat([starts, row_starts]))
                cu = torch.cat([starts, torch.tensor([T], device=dev)]).to(torch.int32)
                max_seqlen = int((cu[1:] - cu[:-1]).max().item())
            else:
                cu = cu_seqlens.to(device=dev, dtype=torch.int32)
                if max_seqlen is None:
                    max_seqlen = int((cu[1:] - cu[:-1]).max().item())
        cp = self.cp_group is not None
        if cp:
            assert position_ids is not None, "context parallel needs the global position_ids (cp_batch)"
            cos, sin = self._rope_tables(int(position_ids.max()) + 1, dev)
        else:
            cos, sin = self._rope_tables(S, dev)
        return RunCtx(cos, sin, pos, cu, int(max_seqlen), self.cp_group if cp else None, B,
                      self.sp_group if sp else None, cp_ranges)

    def embed(self, input_ids):
        ids = input_ids.reshape(-1)
        tp = self.tp
        if tp.enabled:
            x = _VocabParallelEmbedding.apply(ids, self.embed_tokens.weight, self.vocab_start)
            return tp_comm.scatter_seq(x, tp.group)
        return ops.embedding(ids, self.embed_tokens.weight)

    def head(self, x, res, labels=None, num_valid=None, return_logits=False, batch_rows=1):
        """Final norm (with the last residual add) and the fused loss head / logits."""
        tp = self.tp
        h, _ = ops.add_rms_norm(x, res, self.norm.weight, self.config.rms_norm_eps)
        if tp.enabled:
            h = tp_comm.gather_seq(h, tp.group)
        out = CausalLMOutput()
        w = self.lm_head_weight()
        if labels is not None:
            cp, sp = self.cp_group is not None, self.sp_group is not None
            if cp or sp:  # shifted on the full sequence before sharding
                shifted = labels.reshape(-1)
            else:
                shifted = torch.full_like(labels, -100)
                shifted[:, :-1] = labels[:, 1:]
                shifted = shifted.reshape(-1)
            if num_valid is None:
                num_valid = int((shifted != -100).sum().item())
                if cp or sp:  # the loss is a share of the mean over the full rows
                    import torch.distributed as dist

                    t = torch.tensor([num_valid], device=h.device)
                    dist.all_reduce(t, group=self.cp_group if cp else self.sp_group)
                    num_valid = int(t.item())
            if tp.enabled:
                out.loss = ops.vocab_parallel_fused_linear_cross_entropy(
                    h, w, shifted, self.vocab_start, tp.group, num_valid=num_valid)
            else:
                out.loss = ops.fused_linear_cross_entropy(h, w, shifted, num_valid=num_valid)
        if return_logits or labels is None:
            logits = ops.linear(h, w)
            if tp.enabled:
                logits = tp_comm.gather_seq(logits.t().contiguous(), tp.group).t()
            out.logits = logits.view(batch_rows, -1, logits.shape[-1])
        return out


def count_valid_labels(labels: torch.Tensor, ignore_index: int = -100) -> int:
    """Host-side count of shifted labels that contribute to the loss (call on the CPU batch)."""
    return int((labels[:, 1:] != ignore_index).sum())
