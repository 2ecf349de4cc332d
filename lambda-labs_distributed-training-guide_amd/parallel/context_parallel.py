"""Context parallelism for long sequences (SURVEY §2.3 "CP", §5.7 stretch goal).

Each of the `cp` ranks of a context-parallel group holds 1/cp of every sequence, in the
zig-zag layout that balances causal work: a row of S tokens is cut into 2*cp chunks of
c = S / (2*cp) tokens and rank r keeps chunks r and 2*cp-1-r.  Norms, projections, the MLP
and the loss are token-local and run on the local shard unchanged; only attention needs the
other ranks' keys and values:

  forward   all-gather K|V over the group (one RCCL all-gather per layer -- the 8 GPUs of an
            MI355X node are fully connected, so the gather needs no ring of point-to-point
            steps) and put the rows in global order (one index_select); then ONE varlen flash
            call in which every local query chunk g is a sequence whose keys are its row's
            prefix 0 .. (g+1)c, causal mask bottom-right aligned (the kernels' per-sequence key
            ranges).  No per-block launches and no log-sum-exp merge.
  backward  one varlen backward per local chunk slot (the two slots' key prefixes overlap),
            dK / dV of the two added, one index_select back to rank order and one
            reduce-scatter to the owners: O(1) launches per layer in both passes.

Work per rank: the causal work of chunks r and 2cp-1-r, equal on every rank.

Packed rows (several documents per row, 00-rime): a local chunk is cut at the document
boundaries into pieces, and each piece is a varlen "sequence" whose keys are its document's
prefix up to the piece's end (bottom-right causal alignment again) -- attention never crosses a
document, RoPE uses the per-document positions, and the launch count stays O(1) per layer.
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


def cp_batch(input_ids: torch.Tensor, rank: int, cp: int, ignore_index: int = -100, labels=None,
             position_ids=None):
    """Shard a full [B, S] batch for context parallelism.

    Returns (ids, shifted_labels, position_ids, num_valid_total): labels are shifted on the
    FULL sequence first (the next token of a chunk's last token lives on another rank),
    positions are the global ones -- or, for packed rows, the given per-document positions
    (RoPE) -- and num_valid_total is the global label count."""
    B, S = input_ids.shape
    shifted = torch.full_like(input_ids, ignore_index)
    shifted[:, :-1] = (input_ids if labels is None else labels)[:, 1:]
    pos = torch.arange(S, device=input_ids.device).expand(B, S) if position_ids is None else position_ids
    n_valid = int((shifted != ignore_index).sum())
    return (shard_zigzag(input_ids, rank, cp), shard_zigzag(shifted, rank, cp), shard_zigzag(pos, rank, cp), n_valid)


# ------------------------------------------------------------------------------ attention
def _chunk_perm(cp: int, device) -> torch.Tensor:
    """perm[g] = position of global chunk g in the gathered (rank, slot) order."""
    idx = []
    for g in range(2 * cp):
        idx.append(2 * g if g < cp else 2 * (2 * cp - 1 - g) + 1)
    return torch.tensor(idx, dtype=torch.long, device=device)


def _gather_kv(k, v, group, cp, B, c):
    """Local K|V [B*2c, H, D] -> full rows [B*S, H, D] (K and V) in global token order: one
    all-gather and one index_select, no per-chunk copies."""
    kv = torch.cat([k, v], dim=1).contiguous()                      # [B*2c, 2H, D]
    out = comm.all_gather_dim0(kv, group) if cp > 1 else kv          # [cp*B*2c, 2H, D]
    H2, D = kv.shape[1], kv.shape[2]
    rs = out.view(cp, B, 2, c, H2, D).transpose(0, 1).reshape(B, 2 * cp, c, H2, D)  # (rank, slot) order
    full = rs.index_select(1, _chunk_perm(cp, kv.device)).reshape(B * 2 * cp * c, H2, D)
    H = H2 // 2
    return full[:, :H].contiguous(), full[:, H:].contiguous()


def row_doc_starts(cu_seqlens, B: int, S: int):
    """Per-row document start offsets (row coordinates, 0 included) from the flattened [B*S]
    document boundaries of a packed batch (`PackedCollator`'s cu_seqlens)."""
    cu = [int(x) for x in torch.as_tensor(cu_seqlens).tolist()]
    rows = [[0] for _ in range(B)]
    for x in cu:
        b, off = divmod(x, S)
        if b < B and off > 0:
            rows[b].append(off)
    return [sorted(set(r)) for r in rows]


def packed_ranges(rank, cp, B, c, row_docs, device, slots=(0, 1)):
    """Varlen description of the local query chunks of `slots` for packed rows: every (row, slot)
    chunk is cut at document boundaries; a piece is one sequence whose keys are its document's
    prefix in the gathered full rows, up to the piece's last token.  Returns (cu_seqlens_q,
    k_start, k_len, max_q, max_k)."""
    S = 2 * cp * c
    g = zigzag_chunks(rank, cp)
    qlens, starts, lens = [], [], []
    for b in range(B):
        docs = row_docs[b] + [S]
        for s in slots:
            lo, hi = g[s] * c, (g[s] + 1) * c
            for ds, de in zip(docs[:-1], docs[1:]):
                a, e = max(ds, lo), min(de, hi)
                if a < e:
                    qlens.append(e - a)
                    starts.append(b * S + ds)
                    lens.append(e - ds)
    cu = [0]
    for n in qlens:
        cu.append(cu[-1] + n)
    mk = lambda xs: torch.tensor(xs, dtype=torch.int32, device=device)
    return mk(cu), mk(starts), mk(lens), max(qlens), max(lens)


def cp_ranges(rank, cp, B, c, device, row_docs=None):
    """{"all": ranges of both local slots, 0: slot 0, 1: slot 1} for the forward and the two
    per-slot backward calls (dense rows: one sequence per chunk)."""
    if row_docs is None:
        f = lambda sl: _ranges(rank, cp, B, c, device, sl)
        return {k: (*f(sl)[:3], c, f(sl)[3]) for k, sl in (("all", (0, 1)), (0, (0,)), (1, (1,)))}
    return {k: packed_ranges(rank, cp, B, c, row_docs, device, sl) for k, sl in (("all", (0, 1)), (0, (0,)), (1, (1,)))}


def _ranges(rank, cp, B, c, device, slots=(0, 1)):
    """cu_seqlens over the local query chunks of `slots` (one sequence per (row, slot)) and
    each chunk's key range: the prefix of its row up to and including its own chunk."""
    S = 2 * cp * c
    g = zigzag_chunks(rank, cp)
    starts, lens = [], []
    for b in range(B):
        for s in slots:
            starts.append(b * S)
            lens.append((g[s] + 1) * c)
    n = len(starts)
    cu = torch.arange(0, (n + 1) * c, c, dtype=torch.int32, device=device)
    mk = lambda xs: torch.tensor(xs, dtype=torch.int32, device=device)
    return cu, mk(starts), mk(lens), max(lens)


class _CPAttention(torch.autograd.Function):
    """Each local query chunk attends to the causal prefix of its row in ONE varlen flash call
    (per-sequence key ranges, bottom-right causal alignment): no per-block launches, no
    log-sum-exp merge.  Backward: one varlen call per local chunk slot (their key prefixes
    overlap, so dK / dV of the two slots are computed separately and added), then one
    reduce-scatter of the full-row dK|dV to the owners."""

    @staticmethod
    def forward(ctx, q, k, v, group, cp, rank, B, scale, ranges):
        # q [B*2c, Hq, D], k / v [B*2c, Hkv, D] (local zig-zag shard, row-major over rows)
        T, Hq, D = q.shape
        c = T // (2 * B)
        kf, vf = _gather_kv(k, v, group, cp, B, c)
        q = q.contiguous()
        if ranges is None:
            ranges = cp_ranges(rank, cp, B, c, q.device)
        cu, ks, kl, maxq, maxk = ranges["all"]
        out, lse = torch.ops.dtg.flash_attn_varlen_fwd(q, kf, vf, cu, ks, kl, maxq, maxk, scale, True)
        ctx.save_for_backward(q, kf, vf, out, lse)
        ctx.meta = (group, cp, rank, B, c, scale, k.shape[1], ranges)
        return out

    @staticmethod
    def backward(ctx, dout):
        q, kf, vf, out, lse = ctx.saved_tensors
        group, cp, rank, B, c, scale, Hkv, ranges = ctx.meta
        T, Hq, D = q.shape
        sl = lambda t: t.view(B, 2, c, *t.shape[1:])
        q5, o5, do5 = sl(q), sl(out), sl(dout.contiguous())
        lse4 = lse.view(Hq, B, 2, c)
        dq = torch.empty_like(q5)
        dk = dv = None
        for s in (0, 1):
            cu, ks, kl, maxq, maxk = ranges[s]
            flat = lambda t: t[:, s].reshape(B * c, *t.shape[3:])
            dqs, dks, dvs = torch.ops.dtg.flash_attn_varlen_bwd(
                flat(do5), flat(q5), kf, vf, flat(o5), lse4[:, :, s].reshape(Hq, B * c).contiguous(), cu, ks, kl, maxq, maxk,
                scale, True)
            dq[:, s] = dqs.view(B, c, Hq, D)
            dk = dks.float() if dk is None else dk + dks.float()
            dv = dvs.float() if dv is None else dv + dvs.float()
        # full-row dK|dV -> (rank, slot) order -> reduce-scatter to the owners
        S = 2 * cp * c
        dkv = torch.cat([dk, dv], dim=1).to(q.dtype).view(B, 2 * cp, c, 2 * Hkv, D)
        inv = torch.argsort(_chunk_perm(cp, q.device))
        send = dkv.index_select(1, inv).view(B, cp, 2, c, 2 * Hkv, D).transpose(0, 1).reshape(cp * B * 2 * c, 2 * Hkv, D)
        mine = comm.reduce_scatter_dim0(send.contiguous(), group) if cp > 1 else send  # [B*2c, 2Hkv, D]
        return (dq.view(T, Hq, D), mine[:, :Hkv].contiguous(), mine[:, Hkv:].contiguous(),
                None, None, None, None, None, None)


def cp_attention(q, k, v, group, batch_rows: int, scale: float | None = None, ranges=None):
    """Exact causal attention over zig-zag context-parallel shards.

    q [B*S/cp, Hq, D], k / v [B*S/cp, Hkv, D]: this rank's tokens, rows concatenated, each row
    holding its two chunks; returns this rank's attention output [B*S/cp, Hq, D].  `ranges`
    (`cp_ranges(..., row_docs)`) describes packed rows; None = dense rows."""
    cp = comm.world(group) if dist.is_initialized() else 1
    rank = comm.rank(group) if cp > 1 else 0
    if scale is None:
        scale = 1.0 / math.sqrt(q.shape[-1])
    return _CPAttention.apply(q, k, v, group, cp, rank, batch_rows, float(scale), ranges)
