"""Autograd functions for the decoder hot path.

Each function is a thin torch.autograd.Function over `torch.ops.dtg.*` (HIP on GPU, f32
reference on CPU) or hipBLASLt GEMMs (`torch.mm`).  Activations stay 2-D token-major
[T, features] end to end, so no transposes/copies appear between kernels.
"""
import math
import os

import torch
import torch.distributed as dist
import torch.nn.functional as F

from . import grad_routing as _gr
from .grad_routing import route_embedding_grad, route_param_grad, route_weight_grad_mm

ops = torch.ops.dtg


# --------------------------------------------------------------------------------------------
# Linear (hipBLASLt) with direct weight-gradient routing
# --------------------------------------------------------------------------------------------
# Operand layouts of the backward GEMMs.  hipBLASLt's MFMA kernels are fastest when both
# operands are K-contiguous ("TN"); dX = dY W reads W along its strided dim ("NN") and
# dW = dY^T X reduces over the strided token dim of both activations ("NT").  With
# DTG_LINEAR_BWD=tn the backward hands hipBLASLt explicit transposed copies (one streaming
# pass each through csrc/kernels/transpose.hip); "native" keeps the strided forms; "auto"
# transposes W for every dX and dY, X only for dW of layers whose output is at least as wide as
# their input.  Measured on MI355X (Llama-3-8B, b16 x s1024, profiles/r1/s15_*): native 24.0k,
# auto 25.4k, tn 25.4k tok/s; round 2 with every layout's shapes tuned (profiles/r2/s32/bench_*.log):
# native 24.3k, auto 27.0k, tn 27.0-27.1k -- "tn" is the default.
_LINEAR_BWD = os.environ.get("DTG_LINEAR_BWD", "tn")
_TN_MIN_TOKENS = 4096


def _tn_ok(*ts):
    return all(t.is_cuda and t.dtype == torch.bfloat16 and t.shape[0] % 8 == 0 and t.shape[1] % 8 == 0
               and t.stride(1) == 1 for t in ts)


def _wt(w):
    """K-contiguous W^T for dX = dY W: the engine's persistent copy (refreshed by the optimizer
    kernel, parallel/data_parallel.py) when it is current, else a transpose now."""
    ref = getattr(w, "_dtg_wt", None)
    if ref is not None:
        t = ref[0].weight_t(ref[1])
        if t is not None:
            return t
    return ops.transpose2d(w)


def _bwd_layout(x, w):
    """(dx_tn, dw_tn) for this Linear's backward."""
    mode = _LINEAR_BWD
    if mode == "native" or x.shape[0] < _TN_MIN_TOKENS or not _tn_ok(x, w):
        return False, False
    if mode == "tn":
        return True, True
    return True, w.shape[0] >= w.shape[1]


class _Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, out=None):
        ctx.save_for_backward(x, w)
        if out is not None:  # (buffer,): hidden from autograd, e.g. an xGMI workspace slot
            return torch.mm(x, w.t(), out=out[0])
        return torch.mm(x, w.t())

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dx_tn, dw_tn = _bwd_layout(x, w)
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx = torch.mm(dy, _wt(w).t()) if dx_tn else torch.mm(dy, w)
        if ctx.needs_input_grad[1]:
            if dw_tn and _tn_ok(dy):
                dw = route_weight_grad_mm(w, dy, x, a_t=ops.transpose2d(dy), b_t=ops.transpose2d(x))
            else:
                dw = route_weight_grad_mm(w, dy, x)
        return dx, dw, None


def linear(x, w, b=None, out=None):
    """y = x @ w^T (+ b); x is [T, in].  `out`: preallocated [T, out_features] result buffer
    (no bias) -- the zero-copy reduce-scatter input of a tensor-parallel region."""
    if b is None:
        return _Linear.apply(x, w, None if out is None else (out,))
    assert out is None, "linear: out= is for the bias-free projections"
    return _LinearBias.apply(x, w, b)


class _LinearBias(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w, b)
        return torch.addmm(b, x, w.t())

    @staticmethod
    def backward(ctx, dy):
        x, w, b = ctx.saved_tensors
        dx_tn, dw_tn = _bwd_layout(x, w)
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = torch.mm(dy, _wt(w).t()) if dx_tn else torch.mm(dy, w)
        if ctx.needs_input_grad[1]:
            if dw_tn and _tn_ok(dy):
                dw = route_weight_grad_mm(w, dy, x, a_t=ops.transpose2d(dy), b_t=ops.transpose2d(x))
            else:
                dw = route_weight_grad_mm(w, dy, x)
        if ctx.needs_input_grad[2]:
            db = route_param_grad(b, dy.sum(0, dtype=torch.float32).to(dy.dtype))
        return dx, dw, db


# --------------------------------------------------------------------------------------------
# RMSNorm and fused residual-add + RMSNorm
# --------------------------------------------------------------------------------------------
class _RMSNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, eps):
        y, rstd = ops.rmsnorm_fwd(x, w, eps)
        ctx.save_for_backward(x, w, rstd)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, rstd = ctx.saved_tensors
        dx, dw = ops.rmsnorm_bwd(dy, x, w, rstd, None)
        return dx, route_param_grad(w, dw), None


class _AddRMSNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, res, w, eps):
        y, h, rstd = ops.add_rmsnorm_fwd(x, res, w, eps)
        ctx.save_for_backward(h, w, rstd)
        return y, h

    @staticmethod
    def backward(ctx, dy, dh):
        h, w, rstd = ctx.saved_tensors
        if dy is None:
            dy = torch.zeros_like(h)
        dx, dw = ops.rmsnorm_bwd(dy, h, w, rstd, dh)
        return dx, dx, route_param_grad(w, dw), None


def rms_norm(x, w, eps):
    return _RMSNorm.apply(x, w, eps)


def add_rms_norm(x, res, w, eps):
    """Returns (rmsnorm(x + res), x + res)."""
    return _AddRMSNorm.apply(x, res, w, eps)


# --------------------------------------------------------------------------------------------
# Rotary tables
# --------------------------------------------------------------------------------------------
def _llama3_inv_freq(inv_freq, scaling):
    factor = scaling["factor"]
    low = scaling.get("low_freq_factor", 1.0)
    high = scaling.get("high_freq_factor", 4.0)
    old_ctx = scaling["original_max_position_embeddings"]
    low_wl = old_ctx / low
    high_wl = old_ctx / high
    wavelen = 2 * math.pi / inv_freq
    out = torch.where(wavelen > low_wl, inv_freq / factor, inv_freq)
    smooth = (old_ctx / wavelen - low) / (high - low)
    smoothed = (1 - smooth) * out / factor + smooth * out
    is_medium = (wavelen >= high_wl) & (wavelen <= low_wl)
    return torch.where(is_medium, smoothed, out)


def rope_tables(head_dim, theta, max_pos, scaling=None, device=None):
    """cos/sin [max_pos, head_dim/2] f32 (HF LlamaRotaryEmbedding semantics, incl. llama3 scaling)."""
    inv_freq = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.int64).float() / head_dim))
    attn_factor = 1.0
    if scaling is not None:
        kind = scaling.get("rope_type", scaling.get("type"))
        if kind == "llama3":
            inv_freq = _llama3_inv_freq(inv_freq, scaling)
        elif kind in (None, "default"):
            pass
        else:
            raise NotImplementedError(f"rope scaling {kind}")
    t = torch.arange(max_pos, dtype=torch.float32)
    freqs = torch.outer(t, inv_freq)
    cos = (freqs.cos() * attn_factor).contiguous()
    sin = (freqs.sin() * attn_factor).contiguous()
    if device is not None:
        cos, sin = cos.to(device), sin.to(device)
    return cos, sin


# --------------------------------------------------------------------------------------------
# Attention (RoPE fused into the same autograd node; fused QKV in, fused dQKV out)
# --------------------------------------------------------------------------------------------
# The RoPE backward of the q / k heads runs inside the attention backward's dQ / dK epilogues
# (csrc/kernels/flash_attn.hip, one bf16 rounding) instead of a separate in-place pass:
# -1.64 ms of RoPE kernels, +0.78 ms of epilogue per 8B step (profiles/r4/s45).
# DTG_FA_ROPE_FUSED=0 restores the separate pass.
_FA_ROPE_FUSED = os.environ.get("DTG_FA_ROPE_FUSED", "1") == "1"


class _AttentionQKV(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, cos, sin, pos, cu_seqlens, max_seqlen, nq, nkv, head_dim, scale, causal, rope, window):
        T = qkv.shape[0]
        d = head_dim
        if rope:
            ops.rope_(qkv, cos, sin, pos, nq + nkv, d, False)
        q = qkv.as_strided((T, nq, d), (qkv.stride(0), d, 1), qkv.storage_offset())
        k = qkv.as_strided((T, nkv, d), (qkv.stride(0), d, 1), qkv.storage_offset() + nq * d)
        v = qkv.as_strided((T, nkv, d), (qkv.stride(0), d, 1), qkv.storage_offset() + (nq + nkv) * d)
        o, lse = ops.flash_attn_fwd(q, k, v, cu_seqlens, max_seqlen, scale, causal, window)
        ctx.save_for_backward(qkv, o, lse, cu_seqlens, cos, sin, pos)
        ctx.meta = (max_seqlen, nq, nkv, d, scale, causal, rope, window)
        return o.view(T, nq * d)

    @staticmethod
    def backward(ctx, do):
        qkv, o, lse, cu, cos, sin, pos = ctx.saved_tensors
        max_seqlen, nq, nkv, d, scale, causal, rope, window = ctx.meta
        T = qkv.shape[0]
        if rope and _FA_ROPE_FUSED:  # RoPE backward inside the dQ / dK epilogues
            dqkv = ops.flash_attn_bwd_qkv_rope(do.contiguous().view(T, nq, d), qkv, nq, nkv, d, o, lse, cu, max_seqlen,
                                               scale, causal, cos, sin, pos, window)
        else:
            dqkv = ops.flash_attn_bwd_qkv(do.contiguous().view(T, nq, d), qkv, nq, nkv, d, o, lse, cu, max_seqlen,
                                          scale, causal, window)
            if rope:
                ops.rope_(dqkv, cos, sin, pos, nq + nkv, d, True)
        return dqkv, None, None, None, None, None, None, None, None, None, None, None, None


class _AttentionQKVDrop(torch.autograd.Function):
    """Attention with dropout on the probabilities, inside the flash kernels: the keep mask is a
    counter-based (Philox) function of (seed, offset, head, query, key), drawn in the forward and
    regenerated in the backward -- nothing [S, S] is stored.  {seed, offset} is a device tensor
    drawn from torch's CUDA generator (ops.philox_rng), so a captured HIP graph draws a new mask
    every replay (a Python int would be baked into the graph)."""

    @staticmethod
    def forward(ctx, qkv, cu_seqlens, max_seqlen, nq, nkv, head_dim, scale, causal, p, rng):
        T = qkv.shape[0]
        d = head_dim
        q = qkv.as_strided((T, nq, d), (qkv.stride(0), d, 1), qkv.storage_offset())
        k = qkv.as_strided((T, nkv, d), (qkv.stride(0), d, 1), qkv.storage_offset() + nq * d)
        v = qkv.as_strided((T, nkv, d), (qkv.stride(0), d, 1), qkv.storage_offset() + (nq + nkv) * d)
        o, lse = ops.flash_attn_fwd_drop(q, k, v, cu_seqlens, max_seqlen, scale, causal, p, rng)
        ctx.save_for_backward(qkv, o, lse, cu_seqlens, rng)
        ctx.meta = (max_seqlen, nq, nkv, d, scale, causal, p)
        return o.view(T, nq * d)

    @staticmethod
    def backward(ctx, do):
        qkv, o, lse, cu, rng = ctx.saved_tensors
        max_seqlen, nq, nkv, d, scale, causal, p = ctx.meta
        T = qkv.shape[0]
        dqkv = ops.flash_attn_bwd_qkv_drop(do.contiguous().view(T, nq, d), qkv, nq, nkv, d, o, lse, cu, max_seqlen,
                                           scale, causal, p, rng)
        return dqkv, None, None, None, None, None, None, None, None, None


def dropout_rng(like):
    """{seed, offset} (int64 [2] on `like`'s device) of one attention-dropout call: torch's CUDA
    generator on a GPU (graph-safe), its CPU generator on the CPU reference path."""
    return ops.philox_rng(like, 4)


class _Rope(torch.autograd.Function):
    """Out-of-place RoPE on the q and k heads of a fused QKV activation (v untouched)."""

    @staticmethod
    def forward(ctx, qkv, cos, sin, pos, nheads, head_dim):
        y = qkv.contiguous().clone()
        ops.rope_(y, cos, sin, pos, nheads, head_dim, False)
        ctx.save_for_backward(cos, sin, pos)
        ctx.meta = (nheads, head_dim)
        return y

    @staticmethod
    def backward(ctx, dy):
        cos, sin, pos = ctx.saved_tensors
        dx = dy.contiguous().clone()
        ops.rope_(dx, cos, sin, pos, ctx.meta[0], ctx.meta[1], True)
        return dx, None, None, None, None, None


def rope(qkv, cos, sin, pos, nheads, head_dim):
    return _Rope.apply(qkv, cos, sin, pos, int(nheads), int(head_dim))


FA_HEAD_DIMS = (64, 128)  # head dims the flash-attention kernels are instantiated for


def _attention_padded(qkv, nq, nkv, d, cu_seqlens, max_seqlen, cos, sin, pos, causal, scale, window):
    """Head dims without a kernel instantiation (e.g. 80, 96, 48): zero-pad every head to the next
    instantiated width.  Zero columns add nothing to q.k (the scale keeps 1/sqrt(d) of the true
    width) and give zero output columns, which are sliced off; autograd drops their gradients.
    Costs the padded width's FLOPs, not a second code path."""
    dp = next((x for x in FA_HEAD_DIMS if x >= d), None)
    if dp is None or d % 2:
        raise ValueError(f"attention: head_dim {d} unsupported (kernels: {FA_HEAD_DIMS}; smaller even dims are padded)")
    T = qkv.shape[0]
    x = qkv.reshape(T, nq + 2 * nkv, d)
    if cos is not None:  # RoPE out of place in torch (the rope kernel is instantiated for 64/128 too)
        h = d // 2
        qk = x[:, : nq + nkv].float()
        c, s = cos[pos][:, None, :], sin[pos][:, None, :]
        x1, x2 = qk[..., :h], qk[..., h:]
        rot = torch.cat([x1 * c - x2 * s, x2 * c + x1 * s], -1).to(x.dtype)
        x = torch.cat([rot, x[:, nq + nkv:]], 1)
    xp = F.pad(x, (0, dp - d)).reshape(T, (nq + 2 * nkv) * dp)
    e = torch.empty(0, device=qkv.device)
    o = _AttentionQKV.apply(xp, e, e, torch.empty(0, dtype=torch.long, device=qkv.device), cu_seqlens, int(max_seqlen),
                            nq, nkv, dp, float(scale), causal, False, int(window or 0))
    return o.view(T, nq, dp)[..., :d].reshape(T, nq * d)


def attention(qkv, nq, nkv, head_dim, cu_seqlens, max_seqlen, cos=None, sin=None, pos=None, causal=True, scale=None,
              window=0, dropout_p=0.0):
    """Causal (varlen) GQA attention on a fused [T, (nq+2nkv)*d] QKV activation -> [T, nq*d].

    If cos/sin/pos are given, RoPE is applied to q and k first (in place on qkv).  window > 0:
    sliding-window attention (query i sees keys i - window < j <= i; Mistral).  dropout_p > 0:
    dropout on the attention probabilities inside the flash kernels (GPT-2 training)."""
    if scale is None:
        scale = 1.0 / math.sqrt(head_dim)
    if dropout_p > 0.0:
        if cos is not None or window:
            raise ValueError("attention dropout is supported without RoPE / sliding windows (GPT-2)")
        if qkv.is_cuda and head_dim not in FA_HEAD_DIMS:
            raise ValueError(f"attention dropout: head_dim {head_dim} needs a kernel instantiation {FA_HEAD_DIMS}")
        return _AttentionQKVDrop.apply(qkv, cu_seqlens, int(max_seqlen), nq, nkv, head_dim, float(scale), causal,
                                       float(dropout_p), dropout_rng(qkv))
    if qkv.is_cuda and head_dim not in FA_HEAD_DIMS:  # the CPU reference takes any width
        return _attention_padded(qkv, nq, nkv, head_dim, cu_seqlens, max_seqlen, cos, sin, pos, causal, scale, window)
    rope = cos is not None
    if not rope:
        cos = sin = torch.empty(0, device=qkv.device)
        pos = torch.empty(0, dtype=torch.long, device=qkv.device)
    return _AttentionQKV.apply(qkv, cos, sin, pos, cu_seqlens, int(max_seqlen), nq, nkv, head_dim, float(scale), causal, rope,
                               int(window or 0))


# --------------------------------------------------------------------------------------------
# SwiGLU
# --------------------------------------------------------------------------------------------
class _SwiGLU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gu):
        ctx.save_for_backward(gu)
        return ops.swiglu_fwd(gu)

    @staticmethod
    def backward(ctx, dh):
        (gu,) = ctx.saved_tensors
        return ops.swiglu_bwd(dh.contiguous(), gu)


def swiglu(gu):
    return _SwiGLU.apply(gu)


class _SwiGLUMLP(torch.autograd.Function):
    """down(swiglu(x @ W_gu^T)) as one autograd node.

    Saves only x and gu (h = silu(g)*u is recomputed in backward, [T, I] less resident per
    layer).  On the TN path the backward's SwiGLU kernel writes dgu together with dgu^T and h^T,
    the token-contiguous operands of the two weight-gradient GEMMs, so neither needs a separate
    transpose pass; dX GEMMs use transposed weight copies (see _bwd_layout)."""

    @staticmethod
    def forward(ctx, x, w_gu, w_down, out=None):
        gu = torch.mm(x, w_gu.t())
        h = ops.swiglu_fwd(gu)
        ctx.save_for_backward(x, w_gu, w_down, gu)
        if out is not None:
            return torch.mm(h, w_down.t(), out=out[0])
        return torch.mm(h, w_down.t())

    @staticmethod
    def backward(ctx, dy):
        x, w_gu, w_down, gu = ctx.saved_tensors
        dy = dy.contiguous()
        dx_tn, dw_tn = _bwd_layout(x, w_gu)
        fused = dw_tn and _tn_ok(dy, gu) and gu.stride(0) == gu.shape[1]
        dh = torch.mm(dy, _wt(w_down).t()) if dx_tn else torch.mm(dy, w_down)
        if fused:
            dgu, dgu_t, h_t = ops.swiglu_bwd_t(dh, gu)
            del dh
            dw_down = route_weight_grad_mm(w_down, dy, None, a_t=ops.transpose2d(dy), b_t=h_t)
            del h_t
        else:
            h = ops.swiglu_fwd(gu)
            dgu = ops.swiglu_bwd(dh, gu)
            del dh
            dw_down = route_weight_grad_mm(w_down, dy, h)
            del h
        dx = torch.mm(dgu, _wt(w_gu).t()) if dx_tn else torch.mm(dgu, w_gu)
        if fused:
            dw_gu = route_weight_grad_mm(w_gu, dgu, x, a_t=dgu_t, b_t=ops.transpose2d(x))
        else:
            dw_gu = route_weight_grad_mm(w_gu, dgu, x)
        return dx, dw_gu, dw_down, None


def swiglu_mlp(x, w_gu, w_down, out=None):
    """Llama MLP: down_proj(silu(gate(x)) * up(x)) with the fused [gate; up] weight.  `out`: see
    `linear`."""
    return _SwiGLUMLP.apply(x, w_gu, w_down, None if out is None else (out,))


# --------------------------------------------------------------------------------------------
# Embedding
# --------------------------------------------------------------------------------------------
class _Embedding(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, w):
        ctx.save_for_backward(ids)
        ctx.w = w
        return F.embedding(ids, w)

    @staticmethod
    def backward(ctx, dy):
        (ids,) = ctx.saved_tensors
        w = ctx.w
        return None, route_embedding_grad(w, ids, dy.contiguous(), w.shape[0])


def embedding(ids, w):
    return _Embedding.apply(ids, w)


# --------------------------------------------------------------------------------------------
# Fused lm_head + causal-LM cross entropy (chunked; logits never materialised whole)
# --------------------------------------------------------------------------------------------
def _default_chunk(vocab, hidden_rows):
    """Rows per chunk: ~1 GiB of bf16 logits (DTG_CE_CHUNK_GIB), split evenly over the rows
    (16,384 rows x 128,256 vocab -> 4 x 4,096), a multiple of 64 rows (transposable, MFMA-tile
    aligned), >= 1024."""
    gib = float(os.environ.get("DTG_CE_CHUNK_GIB", "1"))
    n = max(1, -(-hidden_rows * max(vocab, 1) // max(1, int(gib * (1 << 29)))))
    per = -(-hidden_rows // n)
    return max(1024, min(hidden_rows, -(-per // 64) * 64))


def _ce_tn(h, w):
    """Use K-contiguous (TN) operands for the loss head's dX / dW GEMMs (see _bwd_layout)."""
    return _LINEAR_BWD != "native" and _tn_ok(h, w)


def _ce_dx(logits, w, w_t, out):
    """out = logits @ w, as logits @ (w^T)^T when a contiguous w^T is given."""
    if w_t is not None:
        torch.mm(logits, w_t.t(), out=out)
    else:
        torch.mm(logits, w, out=out)


class _FusedLinearCE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, w, labels, ignore_index, num_valid, chunk):
        T = h.shape[0]
        need = ctx.needs_input_grad[0] or ctx.needs_input_grad[1]
        scale = 1.0 / max(num_valid, 1)
        loss_sum = torch.zeros((), dtype=torch.float32, device=h.device)
        dh = torch.empty_like(h) if need else None
        want_dw = need and ctx.needs_input_grad[1]
        # direct: dW goes straight into w.main_grad now (engine-owned loss, grad_output == 1)
        direct = want_dw and _gr.direct_loss_grad() and getattr(w, "main_grad", None) is not None
        dw = torch.empty(w.shape, dtype=w.dtype, device=h.device) if (want_dw and not direct) else None
        # A vocabulary that is not a multiple of 8 (GPT-2 50,257, the rime 156,939) leaves every
        # logits row, and the transposed weight, 16-B misaligned: hipBLASLt then drops to slower
        # kernels and the TN layout cannot be used at all.  Pad the weight with zero rows to the
        # next multiple of 8: the padded logits columns are exactly 0, the CE kernel sees only the
        # first V columns (strided view) and leaves the pad at 0, so the GEMMs over the padded K
        # add nothing.  One 1-GB copy per step for the rime head.
        V = w.shape[0]
        pad = (-V) % 8 if (need and h.is_cuda and _LINEAR_BWD != "native" and chunk % 8 == 0
                           and _tn_ok(h)) else 0
        wp = w
        if pad:
            wp = torch.zeros((V + pad, w.shape[1]), dtype=w.dtype, device=w.device)
            wp[:V].copy_(w.detach())
        tn = need and _ce_tn(h, wp) and chunk % 8 == 0
        w_t = (_wt(w) if wp is w else ops.transpose2d(wp)) if (tn and ctx.needs_input_grad[0]) else None
        for s in range(0, T, chunk):
            e = min(T, s + chunk)
            lp = torch.mm(h[s:e], wp.t())
            logits = lp[:, :V] if pad else lp
            rows = ops.ce_fwd_bwd_(logits, labels[s:e], ignore_index, scale, need)
            loss_sum += rows.sum()
            if need:
                _ce_dx(lp, wp, w_t, dh[s:e])
                if direct and tn:
                    _gr.accumulate_mm_into_main_grad(w, logits, h[s:e], a_t=ops.transpose2d(lp)[:V],
                                                     b_t=ops.transpose2d(h[s:e]))
                elif direct:
                    _gr.accumulate_mm_into_main_grad(w, logits, h[s:e])
                elif dw is not None:
                    # f32 accumulate inside the GEMM, one bf16 rounding per chunk
                    if s == 0:
                        torch.mm(logits.t(), h[s:e], out=dw)
                    else:
                        dw.addmm_(logits.t(), h[s:e])
        ctx.save_for_backward(dh, dw)
        ctx.w = w
        ctx.direct = direct
        return loss_sum * scale

    @staticmethod
    def backward(ctx, go):
        dh, dw = ctx.saved_tensors
        w = ctx.w
        if ctx.direct:
            _gr.notify_param(w)
            return dh, None, None, None, None, None
        gdh = (dh * go.to(dh.dtype)) if ctx.needs_input_grad[0] else None
        gdw = route_param_grad(w, dw * go.to(dw.dtype)) if dw is not None else None
        return gdh, gdw, None, None, None, None


def fused_linear_cross_entropy(h, w, labels, ignore_index=-100, num_valid=None, chunk=None):
    """mean CE of softmax(h @ w^T) vs labels over rows with label != ignore_index.

    `labels` are already shifted (label of row i = token i+1).  `num_valid` (host int) avoids a
    device sync; if None it is computed (one sync)."""
    if num_valid is None:
        num_valid = int((labels != ignore_index).sum().item())
    if chunk is None:
        chunk = _default_chunk(w.shape[0], h.shape[0])
    return _FusedLinearCE.apply(h, w, labels, ignore_index, int(num_valid), int(chunk))


class _VocabParallelFusedLinearCE(torch.autograd.Function):
    """lm_head sharded over the vocabulary across `group` (tensor parallel); h is replicated.

    Per chunk: local logits -> per-row (max, sum-exp, target logit) -> ONE all-gather of those
    [3, rows] stats over the TP group -> global log-sum-exp -> local softmax gradient in place
    (SURVEY C12/K13).  The chunk loop is software-pipelined: chunk j's stats all-gather is in
    flight (async, RCCL's stream) while chunk j+1's logits GEMM and stats kernel run, and only
    then does chunk j's gradient pass wait for it -- no collective sits between the GEMMs.  The
    weight gradient uses K-contiguous (TN) operands and, with an engine-owned loss, accumulates
    straight into `main_grad` (no [V/tp, H] temporary).  The returned dh is this rank's
    vocab-shard PARTIAL; the caller's TP-region entry (sequence all-gather, whose backward is a
    reduce-scatter) sums it across ranks."""

    @staticmethod
    def forward(ctx, h, w, labels, ignore_index, num_valid, chunk, vocab_start, group):
        from ..utils import comm as _comm

        T = h.shape[0]
        need = ctx.needs_input_grad[0] or ctx.needs_input_grad[1]
        scale = 1.0 / max(num_valid, 1)
        loss_sum = torch.zeros((), dtype=torch.float32, device=h.device)
        dh = torch.empty_like(h) if need else None
        want_dw = need and ctx.needs_input_grad[1]
        direct = want_dw and _gr.direct_loss_grad() and getattr(w, "main_grad", None) is not None
        dw = torch.empty(w.shape, dtype=w.dtype, device=h.device) if (want_dw and not direct) else None
        tn = need and _ce_tn(h, w) and chunk % 8 == 0 and w.shape[0] % 8 == 0
        w_t = _wt(w) if (tn and ctx.needs_input_grad[0]) else None

        def issue(s, e):
            logits = torch.mm(h[s:e], w.t())
            m, sx, xl = ops.ce_stats(logits, labels[s:e], vocab_start)
            stats, work = _comm.all_gather_stack_async(torch.stack([m, sx, xl]), group)
            return s, e, logits, stats, work

        def finish(s, e, logits, stats, work):
            nonlocal loss_sum
            work.wait()
            gm = stats[:, 0].amax(0)
            sx = (stats[:, 1] * torch.exp(stats[:, 0] - gm)).sum(0)
            lse = gm + torch.log(sx)
            lab = labels[s:e]
            valid = lab != ignore_index
            loss_sum += torch.where(valid, lse - stats[:, 2].sum(0), torch.zeros_like(lse)).sum()
            if not need:
                return
            ops.ce_grad_(logits, lab, lse.contiguous(), vocab_start, ignore_index, scale)
            _ce_dx(logits, w, w_t, dh[s:e])
            if not want_dw:
                return
            a_t = ops.transpose2d(logits) if tn else None
            b_t = ops.transpose2d(h[s:e]) if tn else None
            if direct:
                _gr.accumulate_mm_into_main_grad(w, logits, h[s:e], a_t=a_t, b_t=b_t)
            else:
                lhs, rhs = (a_t, b_t.t()) if tn else (logits.t(), h[s:e])
                if s == 0:  # f32 accumulate inside the GEMM, one bf16 rounding per chunk
                    torch.mm(lhs, rhs, out=dw)
                else:
                    dw.addmm_(lhs, rhs)

        pend = None
        for s in range(0, T, chunk):
            cur = issue(s, min(T, s + chunk))  # GEMM j+1 overlaps the stats gather of chunk j
            if pend is not None:
                finish(*pend)
            pend = cur
        if pend is not None:
            finish(*pend)
        ctx.save_for_backward(dh, dw)
        ctx.w = w
        ctx.direct = direct
        return loss_sum * scale

    @staticmethod
    def backward(ctx, go):
        dh, dw = ctx.saved_tensors
        if ctx.direct:
            _gr.notify_param(ctx.w)
            return dh, None, None, None, None, None, None, None
        gdh = dh * go.to(dh.dtype) if ctx.needs_input_grad[0] else None
        gdw = route_param_grad(ctx.w, dw * go.to(dw.dtype)) if dw is not None else None
        return gdh, gdw, None, None, None, None, None, None


def vocab_parallel_fused_linear_cross_entropy(h, w_local, labels, vocab_start, group, ignore_index=-100,
                                              num_valid=None, chunk=None):
    if num_valid is None:
        num_valid = int((labels != ignore_index).sum().item())
    if chunk is None:
        chunk = _default_chunk(w_local.shape[0], h.shape[0])
    return _VocabParallelFusedLinearCE.apply(h, w_local, labels, ignore_index, int(num_valid), int(chunk),
                                             int(vocab_start), group)
