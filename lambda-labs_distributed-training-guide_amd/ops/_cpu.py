"""CPU implementations of the `dtg` operators (plain PyTorch, f32 math).

They define the numerics the gfx950 kernels are tested against (tests compare a HIP kernel
with these on the same inputs) and they run the CPU plumbing configuration (GPT-2 / tiny
Llama on the build box).  Registered for the CPU dispatch key only.
"""
import math

import torch
import torch.nn.functional as F

from ._schema import LIB

_LOG2E = 1.4426950408889634


def rmsnorm_fwd(x, w, eps):
    xf = x.float()
    rstd = torch.rsqrt(xf.pow(2).mean(-1) + eps)
    n = (xf * rstd[:, None]).to(x.dtype)
    y = (w.float() * n.float()).to(x.dtype)
    return y, rstd


def add_rmsnorm_fwd(x, res, w, eps):
    h = (x.float() + res.float()).to(x.dtype)
    y, rstd = rmsnorm_fwd(h, w, eps)
    return y, h, rstd


def rmsnorm_bwd(dy, x, w, rstd, dres):
    xf, dyf, wf = x.float(), dy.float(), w.float()
    n = xf * rstd[:, None]
    g = dyf * wf
    dot = (g * n).mean(-1, keepdim=True)
    dx = rstd[:, None] * (g - n * dot)
    if dres is not None:
        dx = dx + dres.float()
    dw = (dyf * n.to(x.dtype).float()).sum(0)
    return dx.to(x.dtype), dw.to(w.dtype)


def rope_(qkv, cos, sin, pos, nheads, head_dim, inverse):
    T = qkv.shape[0]
    half = head_dim // 2
    view = qkv[:, : nheads * head_dim].reshape(T, nheads, head_dim)
    x1 = view[..., :half].float()
    x2 = view[..., half:].float()
    c = cos[pos][:, None, :]
    s = sin[pos][:, None, :]
    if inverse:
        s = -s
    o1 = x1 * c - x2 * s
    o2 = x2 * c + x1 * s
    qkv[:, : nheads * head_dim] = torch.cat([o1, o2], dim=-1).to(qkv.dtype).reshape(T, nheads * head_dim)


def swiglu_fwd(gu):
    inter = gu.shape[1] // 2
    g, u = gu[:, :inter].float(), gu[:, inter:].float()
    return (F.silu(g) * u).to(gu.dtype)


def swiglu_bwd(dh, gu):
    inter = gu.shape[1] // 2
    g, u, d = gu[:, :inter].float(), gu[:, inter:].float(), dh.float()
    s = torch.sigmoid(g)
    du = d * g * s
    dg = d * u * s * (1 + g * (1 - s))
    return torch.cat([dg, du], dim=1).to(gu.dtype)


def ce_fwd_bwd_(logits, labels, ignore_index, grad_scale, compute_grad):
    x = logits.float()
    lse = torch.logsumexp(x, dim=-1)
    valid = labels != ignore_index
    safe = torch.where(valid, labels, torch.zeros_like(labels))
    xl = x.gather(1, safe[:, None])[:, 0]
    loss = torch.where(valid, lse - xl, torch.zeros_like(lse))
    if compute_grad:
        g = torch.exp(x - lse[:, None])
        g.scatter_add_(1, safe[:, None], -torch.ones_like(g[:, :1]))
        g = g * grad_scale
        g[~valid] = 0
        logits.copy_(g.to(logits.dtype))
    return loss


def ce_stats(logits, labels, vocab_start):
    x = logits.float()
    m = x.max(-1).values
    s = torch.exp(x - m[:, None]).sum(-1)
    local = labels - vocab_start
    inside = (local >= 0) & (local < x.shape[1])
    xl = x.gather(1, local.clamp(0, x.shape[1] - 1)[:, None])[:, 0]
    return m, s, torch.where(inside, xl, torch.zeros_like(xl))


def ce_grad_(logits, labels, lse, vocab_start, ignore_index, grad_scale):
    x = logits.float()
    g = torch.exp(x - lse[:, None])
    local = labels - vocab_start
    inside = (local >= 0) & (local < x.shape[1])
    onehot = torch.zeros_like(g)
    rows = torch.nonzero(inside).flatten()
    onehot[rows, local[rows]] = 1.0
    g = (g - onehot) * grad_scale
    g[labels == ignore_index] = 0
    logits.copy_(g.to(logits.dtype))


def adamw_t_(p, master, g, m, v, pt, mats, ntiles, lr, beta1, beta2, eps, wd, step, grad_scale, hyper=None,
             tile_cols=64):
    """The HIP kernel's semantics: only the elements of the listed matrices are updated; each
    matrix with a transposed slot gets its new values transposed into `pt`."""
    for off, rows, cols, toff, _ in mats.tolist():
        n = rows * cols
        sl = slice(off, off + n)
        adamw_(p[sl], None if master is None else master[sl], g[sl], m[sl], v[sl], lr, beta1, beta2, eps, wd,
               step, grad_scale, hyper)
        if toff >= 0:
            pt[toff:toff + n].copy_(p[sl].view(rows, cols).t().reshape(-1))


def adamw_(p, master, g, m, v, lr, beta1, beta2, eps, wd, step, grad_scale, hyper=None):
    bc1 = 1 - beta1**step
    bc2 = math.sqrt(1 - beta2**step)
    if hyper is not None:
        lr, bc1, bc2 = (float(x) for x in hyper[:3].tolist())
    pf = master if master is not None else p.float()
    gf = g.float() * grad_scale
    mf, vf = m.float(), v.float()
    pf = pf * (1 - lr * wd)
    mf = mf + (gf - mf) * (1 - beta1)
    vf = vf * beta2 + (1 - beta2) * gf * gf
    pf = pf - (lr / bc1) * mf / (vf.sqrt() / bc2 + eps)
    m.copy_(mf)
    v.copy_(vf)
    if master is not None:
        master.copy_(pf)
    p.copy_(pf)


def _key_ranges(cu_seqlens, k_start=None, k_len=None):
    """[(q0, q1, k0, k1)] per sequence: self-attention by default, else explicit key ranges with
    the bottom-right-aligned causal mask (query i of n_q attends keys <= i + n_k - n_q)."""
    cu = cu_seqlens.tolist()
    out = []
    for i in range(len(cu) - 1):
        a, b = cu[i], cu[i + 1]
        if k_start is None:
            out.append((a, b, a, b))
        else:
            ks, kl = int(k_start[i]), int(k_len[i])
            out.append((a, b, ks, ks + kl))
    return out


def _mask(nq, nk, window=0):
    # True = masked: key j > query i + (nk - nq), or (sliding window) j <= i + (nk - nq) - window
    i = torch.arange(nq)[:, None]
    j = torch.arange(nk)[None, :]
    m = j > i + (nk - nq)
    if window > 0:
        m = m | (j <= i + (nk - nq) - window)
    return m


def _attn_ref(q, k, v, cu_seqlens, scale, causal, k_start=None, k_len=None, window=0):
    """Per-sequence f32 attention; returns o (bf16/in dtype) and lse [Hq, T] (natural log)."""
    T, hq, d = q.shape
    hkv = k.shape[1]
    rep = hq // hkv
    o = torch.zeros(T, hq, d, dtype=torch.float32)
    lse = torch.full((hq, T), float("-inf"), dtype=torch.float32)
    for a, b, ka, kb in _key_ranges(cu_seqlens, k_start, k_len):
        if b <= a:
            continue
        qs = q[a:b].float().transpose(0, 1)  # [hq, s, d]
        ks = k[ka:kb].float().transpose(0, 1).repeat_interleave(rep, 0)
        vs = v[ka:kb].float().transpose(0, 1).repeat_interleave(rep, 0)
        sc = qs @ ks.transpose(1, 2) * scale
        if causal:
            sc = sc.masked_fill(_mask(b - a, kb - ka, window), float("-inf"))
        l_ = torch.logsumexp(sc, -1)
        p = torch.exp(sc - l_[..., None])
        o[a:b] = (p @ vs).transpose(0, 1)
        lse[:, a:b] = l_
    return o, lse


def _check_qkv(t, name, heads, d):
    """check_qkv of csrc/kernels/flash_attn.hip: [T, H, D], contiguous heads, 16-B token stride."""
    if not (t.dim() == 3 and t.shape[1] == heads and t.shape[2] == d and t.stride(2) == 1 and t.stride(1) == d
            and t.stride(0) % 8 == 0):
        raise RuntimeError(f"dtg: {name} must be [T, H, D] with contiguous heads and 16-B aligned token stride")


def _check_attn_inputs(q, k, v):
    _check_qkv(q, "q", q.shape[1], q.shape[2])
    _check_qkv(k, "k", k.shape[1], q.shape[2])
    _check_qkv(v, "v", k.shape[1], q.shape[2])


def flash_attn_fwd(q, k, v, cu_seqlens, max_seqlen, scale, causal, window=0):
    _check_attn_inputs(q, k, v)
    o, lse = _attn_ref(q, k, v, cu_seqlens, scale, causal, window=window)
    return o.to(q.dtype), lse


# ---- attention dropout: the kernels' counter-based keep mask (csrc/kernels/flash_attn.hip DropCfg)
_PHILOX_M = (0xD2511F53, 0xCD9E8D57)
_PHILOX_W = (0x9E3779B9, 0xBB67AE85)


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Philox4x32-10 on numpy uint64 arrays holding 32-bit values (Random123's round function)."""
    import numpy as np

    m32 = np.uint64(0xFFFFFFFF)
    c = [np.asarray(x, dtype=np.uint64) & m32 for x in (c0, c1, c2, c3)]
    k0, k1 = np.uint64(k0) & m32, np.uint64(k1) & m32
    for r in range(10):
        if r:
            k0 = (k0 + np.uint64(_PHILOX_W[0])) & m32
            k1 = (k1 + np.uint64(_PHILOX_W[1])) & m32
        p0 = np.uint64(_PHILOX_M[0]) * c[0]
        p1 = np.uint64(_PHILOX_M[1]) * c[2]
        c = [(p1 >> np.uint64(32)) ^ c[1] ^ k0, p1 & m32, (p0 >> np.uint64(32)) ^ c[3] ^ k1, p0 & m32]
    return c


def dropout_threshold(p):
    """(thr, scale): keep iff random byte < thr; keep probability thr / 256, scale 256 / thr."""
    thr = max(1, min(256, int(round((1.0 - p) * 256.0))))
    return thr, 256.0 / thr


def dropout_keep(seed, offset, head, s0, nq, nk, p):
    """bool [nq, nk]: the keep decision of (query q, key k) of the sequence starting at token s0
    (sequence-relative q, k) for query head `head` -- byte (k & 3) of word (q & 3) of
    Philox4x32-10({k & ~3, s0 + (q & ~3), head, offset lo}, key = {seed lo, seed hi ^ offset hi}).
    The offset's high word goes into the key, so offsets past 2^32 (long runs draw 4 per call)
    never repeat an earlier mask."""
    import numpy as np

    thr, _ = dropout_threshold(p)
    q = np.arange(nq, dtype=np.uint64)[:, None]
    k = np.arange(nk, dtype=np.uint64)[None, :]
    seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    offset = int(offset) & 0xFFFFFFFFFFFFFFFF
    w = philox4x32_10(k & ~np.uint64(3), np.uint64(s0) + (q & ~np.uint64(3)), np.full_like(q, head),
                      np.full_like(q, offset & 0xFFFFFFFF), seed & 0xFFFFFFFF, (seed >> 32) ^ (offset >> 32))
    sel = (q & np.uint64(3)).astype(np.int64)
    word = np.choose(np.broadcast_to(sel, (nq, nk)), [np.broadcast_to(x, (nq, nk)) for x in w])
    byte = (word >> (np.uint64(8) * (k & np.uint64(3)))) & np.uint64(255)
    return torch.from_numpy(byte.astype(np.int64) < thr)


def _drop_masks(cu_seqlens, hq, p, seed, offset):
    out = []
    for a, b, _, _ in _key_ranges(cu_seqlens):
        out.append(torch.stack([dropout_keep(seed, offset, h, a, b - a, b - a, p) for h in range(hq)]) if b > a else None)
    return out


def _rng_pair(rng):
    seed, offset = (int(x) for x in rng.reshape(-1).tolist())
    return seed, offset


def philox_rng(like, increment):
    """{seed, offset} of one dropout call from torch's CPU generator (reproducible under
    torch.manual_seed, checkpointed with the RNG state)."""
    r = torch.randint(0, 2**62, (2,))
    return torch.tensor([int(r[0]), int(r[1] % (2**31))], dtype=torch.int64)


def flash_attn_fwd_drop(q, k, v, cu_seqlens, max_seqlen, scale, causal, p, rng):
    """o = (M o softmax(S) * 256/thr) V per sequence; lse of the undropped softmax."""
    seed, offset = _rng_pair(rng)
    _check_attn_inputs(q, k, v)
    T, hq, d = q.shape
    rep = hq // k.shape[1]
    _, sc_keep = dropout_threshold(p)
    o = torch.zeros(T, hq, d, dtype=torch.float32)
    lse = torch.full((hq, T), float("-inf"), dtype=torch.float32)
    for (a, b, _, _), m in zip(_key_ranges(cu_seqlens), _drop_masks(cu_seqlens, hq, p, seed, offset)):
        if b <= a:
            continue
        qs = q[a:b].float().transpose(0, 1)
        ks = k[a:b].float().transpose(0, 1).repeat_interleave(rep, 0)
        vs = v[a:b].float().transpose(0, 1).repeat_interleave(rep, 0)
        s = qs @ ks.transpose(1, 2) * scale
        if causal:
            s = s.masked_fill(_mask(b - a, b - a), float("-inf"))
        l_ = torch.logsumexp(s, -1)
        pr = torch.exp(s - l_[..., None]) * m * sc_keep
        o[a:b] = (pr @ vs).transpose(0, 1)
        lse[:, a:b] = l_
    return o.to(q.dtype), lse


def flash_attn_bwd_drop(dout, q, k, v, o, lse, cu_seqlens, max_seqlen, scale, causal, p, rng):
    seed, offset = _rng_pair(rng)
    _check_attn_inputs(q, k, v)
    T, hq, d = q.shape
    hkv = k.shape[1]
    rep = hq // hkv
    _, sc_keep = dropout_threshold(p)
    dq = torch.zeros(T, hq, d, dtype=torch.float32)
    dk = torch.zeros(T, hkv, d, dtype=torch.float32)
    dv = torch.zeros(T, hkv, d, dtype=torch.float32)
    for (a, b, _, _), m in zip(_key_ranges(cu_seqlens), _drop_masks(cu_seqlens, hq, p, seed, offset)):
        if b <= a:
            continue
        qs = q[a:b].float().transpose(0, 1)
        ks = k[a:b].float().transpose(0, 1).repeat_interleave(rep, 0)
        vs = v[a:b].float().transpose(0, 1).repeat_interleave(rep, 0)
        dos = dout[a:b].float().transpose(0, 1)
        os_ = o[a:b].float().transpose(0, 1)
        s = qs @ ks.transpose(1, 2) * scale
        if causal:
            s = s.masked_fill(_mask(b - a, b - a), float("-inf"))
        pr = torch.exp(s - lse[:, a:b].float()[..., None])
        z = pr * m * sc_keep
        dvh = z.transpose(1, 2) @ dos
        dpr = (dos @ vs.transpose(1, 2)) * m * sc_keep
        delta = (dos * os_).sum(-1, keepdim=True)
        ds = pr * (dpr - delta)
        dq[a:b] = (ds @ ks * scale).transpose(0, 1)
        dk[a:b] += (ds.transpose(1, 2) @ qs * scale).view(hkv, rep, b - a, d).sum(1).transpose(0, 1)
        dv[a:b] += dvh.view(hkv, rep, b - a, d).sum(1).transpose(0, 1)
    return dq.to(q.dtype), dk.to(k.dtype), dv.to(v.dtype)


def flash_attn_bwd_qkv_drop(dout, qkv, nq, nkv, head_dim, o, lse, cu_seqlens, max_seqlen, scale, causal, p, rng):
    T = qkv.shape[0]
    d = head_dim
    q = qkv[:, : nq * d].reshape(T, nq, d)
    k = qkv[:, nq * d : (nq + nkv) * d].reshape(T, nkv, d)
    v = qkv[:, (nq + nkv) * d :].reshape(T, nkv, d)
    dq, dk, dv = flash_attn_bwd_drop(dout, q, k, v, o, lse, cu_seqlens, max_seqlen, scale, causal, p, rng)
    return torch.cat([dq.reshape(T, -1), dk.reshape(T, -1), dv.reshape(T, -1)], dim=1)


def flash_attn_varlen_fwd(q, k, v, cu_seqlens_q, k_start, k_len, max_seqlen_q, max_seqlen_k, scale, causal):
    _check_attn_inputs(q, k, v)
    o, lse = _attn_ref(q, k, v, cu_seqlens_q, scale, causal, k_start, k_len)
    return o.to(q.dtype), lse


def flash_attn_bwd(dout, q, k, v, o, lse, cu_seqlens, max_seqlen, scale, causal, window=0, k_start=None, k_len=None):
    """The kernel's semantics: P = exp(S*scale - lse) with the GIVEN lse, delta = rowsum(dO*O)
    with the GIVEN o (so a block of a larger softmax -- context parallelism -- gets the
    gradient of the full softmax)."""
    T, hq, d = q.shape
    _check_attn_inputs(q, k, v)
    # the HIP entry point's layout contract (csrc/kernels/flash_attn.hip), checked here too so the
    # CPU suite catches a caller that would only fail on the GPU (the rime --cp path passed a
    # strided per-slot view of the LSE at batch 1)
    if not (lse.dtype == torch.float32 and lse.is_contiguous() and tuple(lse.shape) == (hq, T)):
        raise RuntimeError("dtg: flash_attn_bwd: lse must be f32 [Hq, T]")
    if not (o.is_contiguous() and dout.shape == o.shape and o.shape[0] == T):
        raise RuntimeError("dtg: flash_attn_bwd: o/dout")
    hkv = k.shape[1]
    rep = hq // hkv
    dq = torch.zeros(T, hq, d, dtype=torch.float32)
    dk = torch.zeros(k.shape[0], hkv, d, dtype=torch.float32)
    dv = torch.zeros(k.shape[0], hkv, d, dtype=torch.float32)
    for a, b, ka, kb in _key_ranges(cu_seqlens, k_start, k_len):
        if b <= a:
            continue
        qs = q[a:b].float().transpose(0, 1)                               # [hq, s, d]
        ks = k[ka:kb].float().transpose(0, 1).repeat_interleave(rep, 0)
        vs = v[ka:kb].float().transpose(0, 1).repeat_interleave(rep, 0)
        dos = dout[a:b].float().transpose(0, 1)
        os_ = o[a:b].float().transpose(0, 1)
        sc = qs @ ks.transpose(1, 2) * scale
        if causal:
            sc = sc.masked_fill(_mask(b - a, kb - ka, window), float("-inf"))
        p = torch.exp(sc - lse[:, a:b].float()[..., None])
        dvh = p.transpose(1, 2) @ dos
        dp = dos @ vs.transpose(1, 2)
        delta = (dos * os_).sum(-1, keepdim=True)
        ds = p * (dp - delta)
        dqh = ds @ ks * scale
        dkh = ds.transpose(1, 2) @ qs * scale
        dq[a:b] = dqh.transpose(0, 1)
        dk[ka:kb] += dkh.view(hkv, rep, kb - ka, d).sum(1).transpose(0, 1)
        dv[ka:kb] += dvh.view(hkv, rep, kb - ka, d).sum(1).transpose(0, 1)
    return dq.to(q.dtype), dk.to(k.dtype), dv.to(v.dtype)


def flash_attn_varlen_bwd(dout, q, k, v, o, lse, cu_seqlens_q, k_start, k_len, max_seqlen_q, max_seqlen_k, scale,
                          causal):
    return flash_attn_bwd(dout, q, k, v, o, lse, cu_seqlens_q, max_seqlen_q, scale, causal, 0, k_start, k_len)


def flash_attn_bwd_qkv(dout, qkv, nq, nkv, head_dim, o, lse, cu_seqlens, max_seqlen, scale, causal, window=0):
    T = qkv.shape[0]
    d = head_dim
    q = qkv[:, : nq * d].reshape(T, nq, d)
    k = qkv[:, nq * d : (nq + nkv) * d].reshape(T, nkv, d)
    v = qkv[:, (nq + nkv) * d :].reshape(T, nkv, d)
    dq, dk, dv = flash_attn_bwd(dout, q, k, v, o, lse, cu_seqlens, max_seqlen, scale, causal, window)
    return torch.cat([dq.reshape(T, -1), dk.reshape(T, -1), dv.reshape(T, -1)], dim=1)


def flash_attn_bwd_qkv_rope(dout, qkv, nq, nkv, head_dim, o, lse, cu_seqlens, max_seqlen, scale, causal, cos, sin,
                            pos, window=0):
    dqkv = flash_attn_bwd_qkv(dout, qkv, nq, nkv, head_dim, o, lse, cu_seqlens, max_seqlen, scale, causal, window)
    rope_(dqkv, cos, sin, pos, nq + nkv, head_dim, True)
    return dqkv


def swiglu_bwd_t(dh, gu):
    dgu = swiglu_bwd(dh, gu)
    return dgu, dgu.t().contiguous(), swiglu_fwd(gu).t().contiguous()


def transpose2d(x):
    return x.t().contiguous()


def transpose_mats_(x, out, mats, mats_host, ntiles):
    for so, r, c, do, _t0 in mats_host.tolist():
        out[do:do + r * c].copy_(x[so:so + r * c].view(r, c).t().reshape(-1))


def embedding_bwd_(out, ids, dy):
    """out[id] += sum of dy rows with that id, f32 sums rounded once; ids outside [0, V) skipped."""
    acc = torch.zeros(out.shape, dtype=torch.float32)
    ids = ids.reshape(-1)
    keep = (ids >= 0) & (ids < out.shape[0])
    acc.index_add_(0, ids[keep], dy.reshape(-1, dy.shape[-1])[keep].float())
    out.copy_((out.float() + acc).to(out.dtype))


_TUNING = [0, 64]


def flash_attn_tuning(like, kv_split, kv_qb):
    """CPU: the reference attention has no launch tuning; the knobs are only remembered."""
    old = list(_TUNING)
    if kv_split >= 0:
        _TUNING[0] = int(kv_split)
    if kv_qb >= 0:
        _TUNING[1] = int(kv_qb)
    return old


for _name, _fn in list(globals().items()):
    if _name in (
        "rmsnorm_fwd", "add_rmsnorm_fwd", "rmsnorm_bwd", "rope_", "swiglu_fwd", "swiglu_bwd",
        "ce_fwd_bwd_", "ce_stats", "ce_grad_", "adamw_", "adamw_t_", "flash_attn_fwd", "flash_attn_bwd",
        "flash_attn_bwd_qkv", "transpose2d", "transpose_mats_", "swiglu_bwd_t", "embedding_bwd_", "flash_attn_varlen_fwd",
        "flash_attn_varlen_bwd", "flash_attn_fwd_drop", "flash_attn_bwd_drop", "flash_attn_bwd_qkv_drop", "philox_rng",
        "flash_attn_bwd_qkv_rope", "flash_attn_tuning",
    ):
        LIB.impl(_name, _fn, "CPU")
