"""T0/T1: op semantics on CPU (reference implementations + autograd wrappers vs plain PyTorch)."""
import math

import pytest
import torch
import torch.nn.functional as F

import dtg  # noqa: F401
from dtg import ops
from dtg.data import packed_position_ids

dops = torch.ops.dtg


def _hf_rmsnorm(x, w, eps):
    xf = x.float()
    return w * (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)).to(x.dtype)


def test_rmsnorm_autograd_matches_eager():
    torch.manual_seed(0)
    x = torch.randn(17, 64, dtype=torch.float32, requires_grad=True)
    w = (1 + 0.1 * torch.randn(64)).requires_grad_()
    y = ops.rms_norm(x, w, 1e-5)
    x2, w2 = x.detach().clone().requires_grad_(), w.detach().clone().requires_grad_()
    y2 = _hf_rmsnorm(x2, w2, 1e-5)
    torch.testing.assert_close(y, y2, atol=1e-5, rtol=1e-5)
    g = torch.randn_like(y)
    y.backward(g)
    y2.backward(g)
    torch.testing.assert_close(x.grad, x2.grad, atol=1e-5, rtol=1e-4)
    torch.testing.assert_close(w.grad, w2.grad, atol=1e-5, rtol=1e-4)


def test_add_rmsnorm_autograd():
    torch.manual_seed(0)
    a = torch.randn(9, 32, requires_grad=True)
    r = torch.randn(9, 32, requires_grad=True)
    w = torch.randn(32, requires_grad=True)
    y, h = ops.add_rms_norm(a, r, w, 1e-6)
    loss = (y * torch.randn_like(y)).sum() + (h * torch.randn_like(h)).sum()
    a2, r2, w2 = (t.detach().clone().requires_grad_() for t in (a, r, w))
    torch.manual_seed(1)
    g1, g2 = torch.randn(9, 32), torch.randn(9, 32)
    y, h = ops.add_rms_norm(a, r, w, 1e-6)
    ((y * g1).sum() + (h * g2).sum()).backward()
    h2 = a2 + r2
    y2 = _hf_rmsnorm(h2, w2, 1e-6)
    ((y2 * g1).sum() + (h2 * g2).sum()).backward()
    for t, u in ((a, a2), (r, r2), (w, w2)):
        torch.testing.assert_close(t.grad, u.grad, atol=1e-4, rtol=1e-4)


def test_swiglu_autograd():
    torch.manual_seed(0)
    gu = torch.randn(11, 48, requires_grad=True)
    h = ops.swiglu(gu)
    gu2 = gu.detach().clone().requires_grad_()
    h2 = F.silu(gu2[:, :24]) * gu2[:, 24:]
    torch.testing.assert_close(h, h2)
    g = torch.randn_like(h)
    h.backward(g)
    h2.backward(g)
    torch.testing.assert_close(gu.grad, gu2.grad, atol=1e-5, rtol=1e-5)


def test_rope_tables_match_hf():
    from transformers import LlamaConfig
    from transformers.models.llama.modeling_llama import LlamaRotaryEmbedding

    scaling = {"rope_type": "llama3", "factor": 8.0, "low_freq_factor": 1.0, "high_freq_factor": 4.0,
               "original_max_position_embeddings": 8192}
    cfg = LlamaConfig(hidden_size=512, num_attention_heads=4, head_dim=128, rope_theta=500000.0,
                      rope_scaling=scaling, max_position_embeddings=131072)
    emb = LlamaRotaryEmbedding(cfg)
    pos = torch.arange(0, 3000, 7)[None]
    cos_hf, sin_hf = emb(torch.zeros(1, dtype=torch.float32), pos)
    cos, sin = ops.rope_tables(128, 500000.0, 3000, scaling)
    torch.testing.assert_close(cos[pos[0]], cos_hf[0, :, :64], atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(sin[pos[0]], sin_hf[0, :, :64], atol=1e-5, rtol=1e-5)


def test_rope_inverse_roundtrip():
    torch.manual_seed(0)
    qkv = torch.randn(20, 3 * 64)
    cos, sin = ops.rope_tables(64, 10000.0, 64)
    pos = torch.randint(0, 64, (20,))
    x = qkv.clone()
    dops.rope_(x, cos, sin, pos, 2, 64, False)
    assert not torch.allclose(x[:, :128], qkv[:, :128])
    torch.testing.assert_close(x[:, 128:], qkv[:, 128:])  # v untouched
    dops.rope_(x, cos, sin, pos, 2, 64, True)
    torch.testing.assert_close(x, qkv, atol=1e-5, rtol=1e-5)


@pytest.mark.parametrize("chunk", [7, 64])
def test_fused_linear_ce_matches_cross_entropy(chunk):
    torch.manual_seed(0)
    T, H, V = 40, 16, 97
    h = torch.randn(T, H, requires_grad=True)
    w = torch.randn(V, H, requires_grad=True)
    labels = torch.randint(0, V, (T,))
    labels[::5] = -100
    loss = ops.fused_linear_cross_entropy(h, w, labels, chunk=chunk)
    h2, w2 = h.detach().clone().requires_grad_(), w.detach().clone().requires_grad_()
    loss2 = F.cross_entropy(h2 @ w2.t(), labels, ignore_index=-100)
    torch.testing.assert_close(loss, loss2, atol=1e-5, rtol=1e-5)
    (2 * loss).backward()
    (2 * loss2).backward()
    torch.testing.assert_close(h.grad, h2.grad, atol=1e-5, rtol=1e-4)
    torch.testing.assert_close(w.grad, w2.grad, atol=1e-5, rtol=1e-4)


def test_attention_op_matches_sdpa_varlen_gqa():
    torch.manual_seed(0)
    lens = [5, 17, 10]
    T, hq, hkv, d = sum(lens), 4, 2, 16
    qkv = torch.randn(T, (hq + 2 * hkv) * d, requires_grad=True)
    cu = torch.tensor([0, 5, 22, 32], dtype=torch.int32)
    o = ops.attention(qkv, hq, hkv, d, cu, max(lens))
    qkv2 = qkv.detach().clone().requires_grad_()
    q, k, v = qkv2.split([hq * d, hkv * d, hkv * d], 1)
    outs = []
    for a, b in zip(cu[:-1].tolist(), cu[1:].tolist()):
        qs = q[a:b].view(b - a, hq, d).transpose(0, 1)
        ks = k[a:b].view(b - a, hkv, d).transpose(0, 1).repeat_interleave(hq // hkv, 0)
        vs = v[a:b].view(b - a, hkv, d).transpose(0, 1).repeat_interleave(hq // hkv, 0)
        outs.append(F.scaled_dot_product_attention(qs, ks, vs, is_causal=True).transpose(0, 1).reshape(b - a, hq * d))
    o2 = torch.cat(outs)
    torch.testing.assert_close(o, o2, atol=1e-5, rtol=1e-5)
    g = torch.randn_like(o)
    o.backward(g)
    o2.backward(g)
    torch.testing.assert_close(qkv.grad, qkv2.grad, atol=1e-4, rtol=1e-4)


@pytest.mark.parametrize("d,window", [(48, 0), (80, 0), (96, 5), (112, 0)])
def test_attention_padded_head_dim_matches_direct(d, window):
    """Head dims without a flash-kernel instantiation run zero-padded to 64/128 on the GPU
    (ops.functional._attention_padded): same output and qkv gradient as the unpadded op,
    RoPE included."""
    from dtg.ops.functional import _attention_padded

    torch.manual_seed(0)
    lens = [9, 23]
    T, hq, hkv = sum(lens), 4, 2
    cu = torch.tensor([0, 9, 32], dtype=torch.int32)
    cos, sin = ops.rope_tables(d, 10000.0, 64)
    pos = torch.cat([torch.arange(n) for n in lens])
    qkv = torch.randn(T, (hq + 2 * hkv) * d, requires_grad=True)
    qkv2 = qkv.detach().clone().requires_grad_()
    o = _attention_padded(qkv, hq, hkv, d, cu, max(lens), cos, sin, pos, True, 1 / math.sqrt(d), window)
    o2 = ops.attention(qkv2.clone(), hq, hkv, d, cu, max(lens), cos, sin, pos, window=window)
    torch.testing.assert_close(o, o2, atol=1e-5, rtol=1e-5)
    g = torch.randn_like(o)
    o.backward(g)
    o2.backward(g)
    torch.testing.assert_close(qkv.grad, qkv2.grad, atol=1e-4, rtol=1e-4)


def test_attention_padded_rejects_wide_heads():
    from dtg.ops.functional import _attention_padded

    with pytest.raises(ValueError, match="head_dim 256"):
        _attention_padded(torch.zeros(4, 3 * 256), 1, 1, 256, torch.tensor([0, 4], dtype=torch.int32), 4,
                          None, None, None, True, 0.1, 0)


def test_adamw_cpu_matches_torch_adamw():
    torch.manual_seed(0)
    p = torch.randn(1000)
    g = torch.randn(1000)
    ref = torch.nn.Parameter(p.clone())
    opt = torch.optim.AdamW([ref], lr=1e-2)
    m, v, pp = torch.zeros(1000), torch.zeros(1000), p.clone()
    for step in range(1, 4):
        ref.grad = g.clone()
        opt.step()
        ops.adamw_step(pp, g, m, v, lr=1e-2, step=step)
    torch.testing.assert_close(pp, ref.detach(), atol=1e-6, rtol=1e-5)


def test_packed_position_ids_edge_cases():
    eos = 9
    x = torch.tensor([1, 2, eos, 3, 4, 5, eos, 6])
    pos, lens = packed_position_ids(x, eos)
    assert pos.tolist() == [0, 1, 2, 0, 1, 2, 3, 0]
    assert lens.tolist() == [3, 4, 1]
    # a single EOS (reference crashes here: SURVEY §2.11 #8)
    x = torch.tensor([1, 2, 3, eos])
    pos, lens = packed_position_ids(x, eos)
    assert pos.tolist() == [0, 1, 2, 3] and lens.tolist() == [4]


def test_transpose2d_and_tn_weight_grad_routing():
    """CPU reference of transpose2d and the transposed-operand weight-gradient GEMM path."""
    from dtg.ops.grad_routing import reset_grad_state, route_weight_grad_mm

    torch.manual_seed(0)
    a, b = torch.randn(64, 24), torch.randn(64, 16)
    at = torch.ops.dtg.transpose2d(a)
    assert at.is_contiguous() and torch.equal(at, a.t())
    ref = a.t() @ b
    p = torch.nn.Parameter(torch.zeros(24, 16))
    torch.testing.assert_close(route_weight_grad_mm(p, a, b, a_t=at, b_t=torch.ops.dtg.transpose2d(b)), ref)
    p.main_grad = torch.zeros(24, 16)
    reset_grad_state([p])
    assert route_weight_grad_mm(p, a, b, a_t=at, b_t=b.t().contiguous()) is None
    assert route_weight_grad_mm(p, a, b) is None  # second contribution accumulates
    torch.testing.assert_close(p.main_grad, 2 * ref)


def test_dropout_mask_offset_high_word_is_keyed():
    """The Philox offset's high word enters the key (ADVICE r5 flash_attn.hip:173): an offset past
    2^32 gives a new mask instead of repeating the mask of its low word; offsets below 2^32 keep
    the round-5 masks (key = seed)."""
    import numpy as np

    from dtg.ops import _cpu

    seed, off = 0x123456789AB, 77
    a = _cpu.dropout_keep(seed, off, 0, 0, 64, 64, 0.5)
    b = _cpu.dropout_keep(seed, off + (1 << 32), 0, 0, 64, 64, 0.5)
    assert not torch.equal(a, b)
    q = np.arange(64, dtype=np.uint64)[:, None]
    k = np.arange(64, dtype=np.uint64)[None, :]
    w = _cpu.philox4x32_10(k & ~np.uint64(3), q & ~np.uint64(3), np.full_like(q, 0), np.full_like(q, off),
                           seed & 0xFFFFFFFF, seed >> 32)
    word = np.choose(np.broadcast_to((q & np.uint64(3)).astype(np.int64), (64, 64)),
                     [np.broadcast_to(x, (64, 64)) for x in w])
    byte = (word >> (np.uint64(8) * (k & np.uint64(3)))) & np.uint64(255)
    assert torch.equal(a, torch.from_numpy(byte.astype(np.int64) < _cpu.dropout_threshold(0.5)[0]))
