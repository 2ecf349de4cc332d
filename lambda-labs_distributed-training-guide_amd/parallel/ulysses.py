"""Ulysses sequence parallelism: all-to-all between sequence shards and head shards
(SURVEY §2.3 "Ulysses (all-to-all seq<->head)" stretch row, §5.7 long context).

Each of the `sp` ranks holds a contiguous 1/sp slice of every sequence.  Everything except
attention is token-local and runs on the slice unchanged.  Around attention, one all-to-all
re-partitions the fused QKV activation from "my tokens, all heads" to "all tokens, my heads"
(sp-th of the query heads and the matching key/value heads), the ordinary varlen flash
attention runs on full sequences -- so packed documents (cu_seqlens) work as they do on one
GPU, unlike the zig-zag block scheme in context_parallel.py -- and a second all-to-all brings
the output back to "my tokens, all heads".

Traffic per layer and rank: (q + 2 kv + o) activations x (sp-1)/sp, independent of the
sequence length share, in two all-to-alls; every MI355X pair in a node has its own xGMI link,
so an all-to-all moves over all 7 links at once (a ring collective would use 2).

Head split: rank j gets query heads [j*nq/sp, (j+1)*nq/sp) and kv heads [j*nkv/sp, ...), which
keeps every GQA group on one rank.  When sp > nkv (e.g. 8 ranks, 2 kv heads), kv heads are
replicated sp/nkv times before the exchange; autograd sums their gradients back.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ..utils import comm


class _SeqToHead(torch.autograd.Function):
    """[B, s, sp, C] (my tokens, per-destination head blocks) -> [B, sp*s, C] (all tokens, my block)."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return _seq_to_head(x, group)

    @staticmethod
    def backward(ctx, dy):
        return _head_to_seq(dy, ctx.group), None


class _HeadToSeq(torch.autograd.Function):
    """[B, sp*s, C] (all tokens, my head block) -> [B, s, sp, C] (my tokens, every rank's block)."""

    @staticmethod
    def forward(ctx, y, group):
        ctx.group = group
        return _head_to_seq(y, group)

    @staticmethod
    def backward(ctx, dx):
        return _seq_to_head(dx, ctx.group), None


def _seq_to_head(x, group):
    B, s, sp, C = x.shape
    send = x.permute(2, 0, 1, 3).contiguous()                       # [dst, B, s, C]
    recv = comm.all_to_all_dim0(send.view(sp * B, s, C), group)     # [src (= seq chunk), B, s, C]
    out = x.new_empty(B, sp * s, C)  # a fresh tensor, never a view of recv: attention ropes it in place
    out.view(B, sp, s, C).copy_(recv.view(sp, B, s, C).permute(1, 0, 2, 3))
    return out


def _head_to_seq(y, group):
    sp = comm.world(group)
    B, S, C = y.shape
    s = S // sp
    send = y.view(B, sp, s, C).permute(1, 0, 2, 3).contiguous()     # [dst (= seq chunk), B, s, C]
    recv = comm.all_to_all_dim0(send.view(sp * B, s, C), group)     # [src (= head block), B, s, C]
    return recv.view(sp, B, s, C).permute(1, 2, 0, 3)                # [B, s, sp, C]


def sp_world(group) -> int:
    return comm.world(group) if dist.is_initialized() else 1


def ulysses_attention(qkv, nq, nkv, d, group, batch_rows, cu_seqlens, max_seqlen, cos, sin, pos_full):
    """Causal attention over Ulysses sequence shards.

    qkv: this rank's fused [B*s, (nq + 2 nkv) * d] projection (pre-RoPE); cu_seqlens / max_seqlen /
    pos_full describe the FULL sequences (B rows of sp*s tokens).  Returns [B*s, nq*d]."""
    from ..ops import functional as F

    sp = sp_world(group)
    T, B = qkv.shape[0], batch_rows
    s = T // B
    assert nq % sp == 0, f"Ulysses degree {sp} must divide the query heads ({nq})"
    q = qkv[:, :nq * d].view(B, s, sp, nq // sp * d)
    k = qkv[:, nq * d:(nq + nkv) * d].view(T, nkv, d)
    v = qkv[:, (nq + nkv) * d:].view(T, nkv, d)
    if nkv % sp:
        assert sp % nkv == 0, f"Ulysses degree {sp} and kv heads {nkv}: one must divide the other"
        r = sp // nkv
        k, v = k.repeat_interleave(r, dim=1), v.repeat_interleave(r, dim=1)
    kvl = k.shape[1] // sp                                          # kv heads per rank
    k = k.reshape(B, s, sp, kvl * d)
    v = v.reshape(B, s, sp, kvl * d)
    x = torch.cat([q, k, v], dim=3)                                 # per-rank fused [q | k | v] blocks
    full = _SeqToHead.apply(x, group)                               # [B, S, C]
    nql = nq // sp
    o = F.attention(full.reshape(B * s * sp, -1), nql, kvl, d, cu_seqlens, max_seqlen, cos, sin, pos_full)
    back = _HeadToSeq.apply(o.view(B, s * sp, nql * d), group)      # [B, s, sp, nql*d]
    return back.reshape(T, nq * d)


def ulysses_batch(input_ids: torch.Tensor, rank: int, sp: int, position_ids=None, ignore_index: int = -100,
                  labels=None):
    """Shard full [B, S] rows for Ulysses: contiguous slices of S/sp tokens.

    Returns (ids, shifted_labels, position_ids or None, num_valid_total); labels are shifted
    on the full rows first (a slice's last token predicts the next slice's first)."""
    B, S = input_ids.shape
    assert S % sp == 0, f"sequence length {S} must divide by the Ulysses degree {sp}"
    s = S // sp
    shifted = torch.full_like(input_ids, ignore_index)
    # same labels as the unsharded model (packed rows included)
    shifted[:, :-1] = (input_ids if labels is None else labels)[:, 1:]
    n_valid = int((shifted != ignore_index).sum())
    sl = slice(rank * s, (rank + 1) * s)
    pos = None if position_ids is None else position_ids[:, sl]
    return input_ids[:, sl], shifted[:, sl], pos, n_valid
