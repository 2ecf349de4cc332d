"""Context parallelism for long sequences (SURVEY §2.3 "CP", §5.7 stretch goal).

Each of the `cp` ranks of a context-parallel group holds 1/cp of every sequence, in the
zig-zag layout that balances causal work: a row of S tokens is cut into 2*cp chunks of
c = S / (2*cp) tokens and rank r keeps chunks r and 2*cp-1-r.  Norms, projections, the MLP
and the loss are token-local and run on the local shard unchanged; only attention needs the
other ranks' keys and values:

  forward   start the all-gather of K|V over the group (one asynchronous RCCL all-gather per
            layer -- the 8 GPUs of an MI355X node are fully connected, so the gather needs no
            ring of point-to-point steps) and, while it is in flight, run the DIAGONAL blocks:
            every local query chunk against its own keys (causal), from the local K/V.  Then put
            the gathered rows in global order (one index_select) and run the OFF-DIAGONAL part:
            every local chunk g against its row's strict prefix 0 .. g*c (no mask).  The two
            partial softmaxes are merged by their log-sum-exps (one elementwise pass).
  backward  off-diagonal: one varlen backward per local chunk slot (the two slots' key
            prefixes overlap), dK / dV of the two added in f32, one index_select back to rank
            order and one f32 reduce-scatter to the owners -- issued asynchronously, and the
            diagonal blocks' backward runs while it is in flight.  O(1) launches per layer in
            both passes; both parts use the MERGED out / lse, so each gets the gradient of the
            full softmax.

Work per rank: the causal work of chunks r and 2cp-1-r, equal on every rank.

Packed rows (several documents per row, 00-rime): a local chunk is cut at the document
boundaries into pieces; a piece's diagonal keys are the piece itself and its off-diagonal keys
its document's part before the chunk (empty if the document starts inside the chunk) --
attention never crosses a document, RoPE uses the per-document positions, and the launch count
stays O(1) per layer.  The varlen descriptions are built ON THE DEVICE from the collator's
cu_seqlens (`cp_ranges`): one entry per (document, local chunk) -- zero-length where they do not
meet -- so nothing is copied to the host and no forward synchronises.
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


def row_doc_starts(cu_seqlens, B: int, S: int):
    """Per-row document start offsets (row coordinates, 0 included) from the flattened [B*S]
    document boundaries of a packed batch (host lists; diagnostics and tests)."""
    cu = [int(x) for x in torch.as_tensor(cu_seqlens).tolist()]
    rows = [[0] for _ in range(B)]
    for x in cu:
        b, off = divmod(x, S)
        if b < B and off > 0:
            rows[b].append(off)
    return [sorted(set(r)) for r in rows]


def packed_ranges(rank, cp, B, c, row_docs, device, slots=(0, 1)):
    """Host reference of the single-call layout (query piece -> its document's prefix up to the
    piece's end, bottom-right causal): (cu_seqlens_q, k_start, k_len, max_q, max_k) without
    empty pieces.  Kept for tests and diagnostics; training uses `cp_ranges`."""
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


_RANGE_CACHE = {}


def cp_ranges(rank, cp, B, c, device, row_docs=None, cu_seqlens=None):
    """Device-side varlen descriptions of this rank's local query chunks (no host sync).

    Documents come from `cu_seqlens` (the collator's flattened [B*S] boundaries, row starts
    included), or host `row_docs` (per-row document starts), or -- both None -- one document
    per row (dense).  Every (document, local chunk) pair is one entry (zero-length when they do
    not meet).  Returns a dict of (cu_seqlens_q, k_start, k_len, max_q, max_k) int32 tuples:
      "diag"     both slots, rows in local (row, slot) order; keys = the piece itself in the LOCAL
                 K/V (causal);
      "off"      same queries; keys = the document's part before the chunk in the GATHERED full
                 rows (no mask; length 0 when the document starts inside the chunk);
      "off0/1"   the off-diagonal part of one slot, rows in that slot's (row) order (backward)."""
    S = 2 * cp * c
    dense = cu_seqlens is None and row_docs is None
    key = (rank, cp, B, c, str(device)) if dense else None
    if key is not None and key in _RANGE_CACHE:
        return _RANGE_CACHE[key]
    if cu_seqlens is not None:
        cu = cu_seqlens.to(device=device, dtype=torch.long)
    elif row_docs is not None:
        cu = torch.tensor([b * S + d for b in range(B) for d in row_docs[b]] + [B * S], dtype=torch.long, device=device)
    else:
        cu = torch.arange(0, (B + 1) * S, S, dtype=torch.long, device=device)
    b = cu[:-1] // S
    ds, de = cu[:-1] - b * S, cu[1:] - b * S  # row-local document spans (documents never cross rows)
    g = zigzag_chunks(rank, cp)
    per = []
    for s in (0, 1):
        lo = g[s] * c
        a = torch.clamp(ds, min=lo)
        qlen = torch.clamp(torch.clamp(de, max=lo + c) - a, min=0)
        ks_diag = (2 * b + s) * c + torch.clamp(a - lo, 0, c)
        kl_off = torch.where(qlen > 0, torch.clamp(lo - ds, min=0), torch.zeros_like(qlen))
        per.append((qlen, ks_diag, b * S + ds, kl_off))
    i32 = lambda t: t.to(torch.int32).contiguous()

    def cu_of(qlen):
        return i32(torch.cat([torch.zeros(1, dtype=torch.long, device=device), torch.cumsum(qlen, 0)]))

    # both slots in local (row, slot, document) order: a stable sort by 2*row + slot
    order = torch.sort(torch.cat([2 * b, 2 * b + 1]), stable=True).indices
    cat = lambda j: torch.cat([per[0][j], per[1][j]])[order]
    qlen_all = cat(0)
    out = {
        "diag": (cu_of(qlen_all), i32(cat(1)), i32(qlen_all), c, c),
        "off": (cu_of(qlen_all), i32(cat(2)), i32(cat(3)), c, S),
    }
    for s in (0, 1):
        qlen, _, ks_off, kl_off = per[s]
        out[f"off{s}"] = (cu_of(qlen), i32(ks_off), i32(kl_off), c, S)
    if key is not None:
        _RANGE_CACHE[key] = out
    return out


def _merge(o_a, lse_a, o_b, lse_b):
    """Two partial softmax attentions over disjoint key sets -> the attention over their union."""
    lse = torch.logaddexp(lse_a, lse_b)                       # [Hq, T]
    wa = torch.exp(lse_a - lse).t().unsqueeze(-1)             # [T, Hq, 1]
    wb = torch.exp(lse_b - lse).t().unsqueeze(-1)
    o = (o_a.float() * wa + o_b.float() * wb).to(o_a.dtype)
    return o.contiguous(), lse.contiguous()


def _order_full(gathered, cp, B, c):
    """Gathered K|V [cp*B*2c, 2H, D] in (rank, slot) order -> full rows [B*S, 2H, D]."""
    H2, D = gathered.shape[1], gathered.shape[2]
    rs = gathered.view(cp, B, 2, c, H2, D).transpose(0, 1).reshape(B, 2 * cp, c, H2, D)
    return rs.index_select(1, _chunk_perm(cp, gathered.device)).reshape(B * 2 * cp * c, H2, D)


class _CPAttention(torch.autograd.Function):
    """Diagonal blocks (local K/V, overlapped with the K/V all-gather) + off-diagonal prefixes
    (gathered K/V) in two varlen flash calls, merged by log-sum-exp; see the module docstring."""

    @staticmethod
    def forward(ctx, q, k, v, group, cp, rank, B, scale, ranges):
        # q [B*2c, Hq, D], k / v [B*2c, Hkv, D] (local zig-zag shard, row-major over rows)
        T, Hq, D = q.shape
        Hkv = k.shape[1]
        c = T // (2 * B)
        kv = torch.cat([k, v], dim=1).contiguous()  # [B*2c, 2Hkv, D]
        if cp > 1:
            gathered = torch.empty((cp * T,) + tuple(kv.shape[1:]), dtype=kv.dtype, device=kv.device)
            work = comm.all_gather_dim0_into_async(gathered, kv, group)
        q = q.contiguous()
        if ranges is None:
            ranges = cp_ranges(rank, cp, B, c, q.device)
        kl_, vl_ = kv[:, :Hkv], kv[:, Hkv:]
        o_a, lse_a = torch.ops.dtg.flash_attn_varlen_fwd(q, kl_, vl_, *ranges["diag"], scale, True)
        if cp > 1:
            work.wait()
            full = _order_full(gathered, cp, B, c)
            del gathered
        else:
            full = kv
        kf, vf = full[:, :Hkv], full[:, Hkv:]
        o_b, lse_b = torch.ops.dtg.flash_attn_varlen_fwd(q, kf, vf, *ranges["off"], scale, False)
        out, lse = _merge(o_a, lse_a, o_b, lse_b)
        ctx.save_for_backward(q, kv, full, out, lse)
        ctx.meta = (group, cp, rank, B, c, scale, Hkv, ranges)
        return out

    @staticmethod
    def backward(ctx, dout):
        q, kv, full, out, lse = ctx.saved_tensors
        group, cp, rank, B, c, scale, Hkv, ranges = ctx.meta
        T, Hq, D = q.shape
        dout = dout.contiguous()
        kf, vf = full[:, :Hkv], full[:, Hkv:]
        sl = lambda t: t.view(B, 2, c, *t.shape[1:])
        q5, o5, do5 = sl(q), sl(out), sl(dout)
        lse4 = lse.view(Hq, B, 2, c)
        dq_b = torch.empty((B, 2, c, Hq, D), dtype=torch.float32, device=q.device)
        dk = dv = None
        for s in (0, 1):  # off-diagonal: the two slots' key prefixes overlap -> one call each
            flat = lambda t: t[:, s].reshape(B * c, *t.shape[3:])
            dqs, dks, dvs = torch.ops.dtg.flash_attn_varlen_bwd(
                flat(do5), flat(q5), kf, vf, flat(o5), lse4[:, :, s].reshape(Hq, B * c).contiguous(),
                *ranges[f"off{s}"], scale, False)
            dq_b[:, s] = dqs.view(B, c, Hq, D).float()
            dk = dks.float() if dk is None else dk + dks.float()
            dv = dvs.float() if dv is None else dv + dvs.float()
        # full-row dK|dV (f32) -> (rank, slot) order -> reduce-scatter to the owners, in flight
        # while the diagonal blocks' backward runs
        dkv = torch.cat([dk, dv], dim=1).view(B, 2 * cp, c, 2 * Hkv, D)
        del dk, dv
        inv = torch.argsort(_chunk_perm(cp, q.device))
        send = dkv.index_select(1, inv).view(B, cp, 2, c, 2 * Hkv, D).transpose(0, 1).reshape(cp * T, 2 * Hkv, D)
        if cp > 1:
            mine = torch.empty((T, 2 * Hkv, D), dtype=torch.float32, device=q.device)
            work = comm.reduce_scatter_dim0_into_async(mine, send.contiguous(), group)
        else:
            mine, work = send, None
        dq_a, dk_a, dv_a = torch.ops.dtg.flash_attn_varlen_bwd(dout, q, kv[:, :Hkv], kv[:, Hkv:], out, lse,
                                                               *ranges["diag"], scale, True)
        if work is not None:
            work.wait()
        dq = (dq_a.float() + dq_b.view(T, Hq, D)).to(q.dtype)
        dk = (dk_a.float() + mine[:, :Hkv]).to(q.dtype)
        dv = (dv_a.float() + mine[:, Hkv:]).to(q.dtype)
        return dq, dk, dv, None, None, None, None, None, None


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
