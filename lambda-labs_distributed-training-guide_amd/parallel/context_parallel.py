"""Context parallelism for long sequences (SURVEY §2.3 "CP", §5.7 stretch goal).

Each of the `cp` ranks of a context-parallel group holds 1/cp of every sequence, in the
zig-zag layout that balances causal work: a row of S tokens is cut into 2*cp chunks of
c = S / (2*cp) tokens and rank r keeps chunks r and 2*cp-1-r.  Norms, projections, the MLP
and the loss are token-local and run on the local shard unchanged; only attention needs the
other ranks' keys and values:

  forward   all-gather K|V over the group (one RCCL all-gather per layer -- the 8 GPUs of an
            MI355X node are fully connected, so the gather needs no ring of point-to-point
            steps), then every local query chunk g attends to key chunks 0..g: the diagonal
            chunk causally, the earlier ones fully.  All (query chunk, key chunk) blocks are
            c x c, so they batch into two varlen flash-attention launches (one causal, one
            not) and the partial outputs merge exactly through their log-sum-exps.
  backward  the same blocks through the flash backward with the MERGED lse and output (so
            every block's softmax and delta = rowsum(dO * O) are the global ones): dQ sums
            over a query's blocks locally; dK / dV blocks accumulate into the full-sequence
            buffers and are reduce-scattered back to their owners.

Work per rank: 2*cp + 1 blocks of c x c, equal on every rank.  Dense rows only (packed
documents would need block masks per document).
"""
from __future__ import annotations

import math
from typing import List, Tuple

import torch
import torch.distributed as dist

from ..utils import comm


# ------------------------------------------------------------------------------ layout
def zigzag_chunks(rank: int, cp: int) -> Tuple[int, int]:
    return rank, 2 * cp - 1 - rank


def shard_zigzag(x: torch.Tensor, rank: int, cp: int) -> torch.Tensor:
    """[B, S, ...] -> this rank's [B, S/cp, ...] (chunks r and 2cp-1-r of every row)."""
    B, S = x.shape[:2]
    assert S % (2 * cp) == 0, f"sequence length {S} must divide by 2*cp={2 * cp}"
    c = S // (2 * cp)
    a, b = zigzag_chunks(rank, cp)
    return torch.cat([x[:, a * c:(a + 1) * c], x[:, b * c:(b + 1) * c]], dim=1)


def unshard_zigzag(shards: List[torch.Tensor], cp: int) -> torch.Tensor:
    """Inverse of shard_zigzag over all ranks' shards (rank order) -> [B, S, ...]."""
    B, half2 = shards[0].shape[:2]
    c = half2 // 2
    chunks = [None] * (2 * cp)
    for r, s in enumerate(shards):
        a, b = zigzag_chunks(r, cp)
        chunks[a], chunks[b] = s[:, :c], s[:, c:]
    return torch.cat(chunks, dim=1)


def cp_batch(input_ids: torch.Tensor, rank: int, cp: int, ignore_index: int = -100, labels=None):
    """Shard a full [B, S] batch for context parallelism.

    Returns (ids, shifted_labels, position_ids, num_valid_total): labels are shifted on the
    FULL sequence first (the next token of a chunk's last token lives on another rank),
    positions are the global ones (RoPE), and num_valid_total is the global label count."""
    B, S = input_ids.shape
    shifted = torch.full_like(input_ids, ignore_index)
    shifted[:, :-1] = (input_ids if labels is None else labels)[:, 1:]
    pos = torch.arange(S, device=input_ids.device).expand(B, S)
    n_valid = int((shifted != ignore_index).sum())
    return (shard_zigzag(input_ids, rank, cp), shard_zigzag(shifted, rank, cp), shard_zigzag(pos, rank, cp), n_valid)


# ------------------------------------------------------------------------------ attention
def _blocks(rank: int, cp: int, B: int):
    """(row, local slot, global query chunk, key chunk) of every c x c block this rank computes."""
    diag, off = [], []
    for b in range(B):
        for slot, gq in enumerate(zigzag_chunks(rank, cp)):
            diag.append((b, slot, gq, gq))
            off.extend((b, slot, gq, j) for j in range(gq))
    return diag, off


def _gather_kv(k, v, group, cp, B, c):
    """Local K|V [B*2c, H, D] -> full-sequence K, V [B, 2cp, c, H, D] in global chunk order."""
    kv = torch.cat([k, v], dim=1).contiguous()                      # [B*2c, 2H, D]
    out = comm.all_gather_dim0(kv, group) if cp > 1 else kv          # [cp*B*2c, 2H, D]
    H2, D = kv.shape[1], kv.shape[2]
    out = out.view(cp, B, 2, c, H2, D)
    full = out.new_empty(B, 2 * cp, c, H2, D)
    for r in range(cp):
        a, bb = zigzag_chunks(r, cp)
        full[:, a] = out[r, :, 0]
        full[:, bb] = out[r, :, 1]
    H = H2 // 2
    return full[..., :H, :], full[..., H:, :]


def _stack(blocks, q, kf, vf):
    """Concatenate the blocks' q / k / v as varlen sequences of c tokens each."""
    qs = torch.stack([q[b, s] for b, s, _, _ in blocks])            # [n, c, Hq, D]
    ks = torch.stack([kf[b, j] for b, _, _, j in blocks])
    vs = torch.stack([vf[b, j] for b, _, _, j in blocks])
    n, c = qs.shape[:2]
    flat = lambda t: t.reshape(n * c, *t.shape[2:])
    cu = torch.arange(0, (n + 1) * c, c, dtype=torch.int32, device=q.device)
    return flat(qs), flat(ks), flat(vs), cu


class _CPAttention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, group, cp, rank, B, scale):
        # q [B*2c, Hq, D], k / v [B*2c, Hkv, D] (local zig-zag shard, row-major over rows)
        T, Hq, D = q.shape
        c = T // (2 * B)
        kf, vf = _gather_kv(k, v, group, cp, B, c)
        q = q.contiguous()
        q5 = q.view(B, 2, c, Hq, D)
        diag, off = _blocks(rank, cp, B)
        ops = torch.ops.dtg
        parts = []  # per block list: (o [c,Hq,D], lse [Hq,c])
        for blocks, causal in ((diag, True), (off, False)):
            if not blocks:
                continue
            qs, ks, vs, cu = _stack(blocks, q5, kf, vf)
            o, lse = ops.flash_attn_fwd(qs, ks, vs, cu, c, scale, causal)
            n = len(blocks)
            parts.append((blocks, o.view(n, c, Hq, D), lse.view(Hq, n, c)))
        # merge the blocks of each (row, slot) through their log-sum-exps
        lse_all = q.new_full((B, 2, Hq, c), -math.inf, dtype=torch.float32)
        for blocks, o, lse in parts:
            for i, (b, s, _, _) in enumerate(blocks):
                lse_all[b, s] = torch.logaddexp(lse_all[b, s], lse[:, i])
        out = torch.zeros(B, 2, c, Hq, D, dtype=torch.float32, device=q.device)
        for blocks, o, lse in parts:
            for i, (b, s, _, _) in enumerate(blocks):
                w = torch.exp(lse[:, i] - lse_all[b, s]).transpose(0, 1).unsqueeze(-1)  # [c, Hq, 1]
                out[b, s] += w * o[i].float()
        out = out.to(q.dtype).view(T, Hq, D)
        ctx.save_for_backward(q, kf, vf, out, lse_all)
        ctx.meta = (group, cp, rank, B, c, scale, k.shape[1])
        return out

    @staticmethod
    def backward(ctx, dout):
        q, kf, vf, out, lse_all = ctx.saved_tensors
        group, cp, rank, B, c, scale, Hkv = ctx.meta
        T, Hq, D = q.shape
        q5 = q.view(B, 2, c, Hq, D)
        o5 = out.view(B, 2, c, Hq, D)
        do5 = dout.contiguous().view(B, 2, c, Hq, D)
        diag, off = _blocks(rank, cp, B)
        ops = torch.ops.dtg
        dq = torch.zeros(B, 2, c, Hq, D, dtype=torch.float32, device=q.device)
        dkf = torch.zeros(kf.shape, dtype=torch.float32, device=q.device)
        dvf = torch.zeros(vf.shape, dtype=torch.float32, device=q.device)
        for blocks, causal in ((diag, True), (off, False)):
            if not blocks:
                continue
            qs, ks, vs, cu = _stack(blocks, q5, kf, vf)
            n = len(blocks)
            os_ = torch.stack([o5[b, s] for b, s, _, _ in blocks]).reshape(n * c, Hq, D)
            dos = torch.stack([do5[b, s] for b, s, _, _ in blocks]).reshape(n * c, Hq, D)
            lse = torch.stack([lse_all[b, s] for b, s, _, _ in blocks], 1).reshape(Hq, n * c).contiguous()
            dqs, dks, dvs = ops.flash_attn_bwd(dos, qs, ks, vs, os_, lse, cu, c, scale, causal)
            dqs, dks, dvs = (t.view(n, c, *t.shape[1:]) for t in (dqs, dks, dvs))
            for i, (b, s, _, j) in enumerate(blocks):
                dq[b, s] += dqs[i].float()
                dkf[b, j] += dks[i].float()
                dvf[b, j] += dvs[i].float()
        # full-sequence dK / dV -> owners: back to [cp, B, 2, c, ...] rank order, reduce-scatter
        dkv = torch.cat([dkf, dvf], dim=3)                                 # [B, 2cp, c, 2Hkv, D]
        send = dkv.new_empty(cp, B, 2, c, 2 * Hkv, D)
        for r in range(cp):
            a, bb = zigzag_chunks(r, cp)
            send[r, :, 0] = dkv[:, a]
            send[r, :, 1] = dkv[:, bb]
        send = send.view(cp * B * 2 * c, 2 * Hkv, D)
        mine = comm.reduce_scatter_dim0(send, group) if cp > 1 else send  # [B*2c, 2Hkv, D]
        dk, dv = mine[:, :Hkv], mine[:, Hkv:]
        return (dq.to(q.dtype).view(T, Hq, D), dk.to(q.dtype).contiguous(), dv.to(q.dtype).contiguous(),
                None, None, None, None, None)


def cp_attention(q, k, v, group, batch_rows: int, scale: float | None = None):
    """Exact causal attention over zig-zag context-parallel shards.

    q [B*S/cp, Hq, D], k / v [B*S/cp, Hkv, D]: this rank's tokens, rows concatenated, each row
    holding its two chunks; returns this rank's attention output [B*S/cp, Hq, D]."""
    cp = comm.world(group) if dist.is_initialized() else 1
    rank = comm.rank(group) if cp > 1 else 0
    if scale is None:
        scale = 1.0 / math.sqrt(q.shape[-1])
    return _CPAttention.apply(q, k, v, group, cp, rank, batch_rows, float(scale))
