"""RoPE backward fused into the flash-attention backward's dQ / dK epilogues
(torch.ops.dtg.flash_attn_bwd_qkv_rope, csrc/kernels/flash_attn.hip) against the unfused path
(flash_attn_bwd_qkv, then rope_(inverse) on the q / k heads): causal and not, GQA, head_dim 128
and 64, packed documents whose positions restart, and the split dK / dV path (f32 partials; the
rotation then runs after the combine)."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


def _tables(max_pos, d):
    inv = 1.0 / (10000.0 ** (torch.arange(0, d, 2, dtype=torch.float64) / d))
    f = torch.outer(torch.arange(max_pos, dtype=torch.float64), inv)
    return f.cos().float().contiguous(), f.sin().float().contiguous()


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


@pytest.mark.parametrize("D,hq,hkv,causal,docs,split,window", [
    (128, 8, 2, True, [0, 512], 1, 0),
    (128, 8, 2, True, [0, 200, 384, 512], 1, 0),
    (128, 4, 1, False, [0, 256, 512], 1, 0),
    (64, 6, 2, True, [0, 300, 512], 1, 0),
    (128, 4, 1, True, [0, 512], 2, 0),
    # sliding window (Mistral) goes through the same epilogues
    (128, 8, 2, True, [0, 512], 1, 128),
    (64, 6, 2, True, [0, 300, 512], 1, 100),
])
def test_fused_rope_bwd_matches_separate_pass(cuda, D, hq, hkv, causal, docs, split, window):
    import dtg.ops

    with dtg.ops.fa_tuning(cuda, kv_split=split):
        _fused_case(cuda, D, hq, hkv, causal, docs, window)


def _fused_case(cuda, D, hq, hkv, causal, docs, window):
    ops = torch.ops.dtg
    torch.manual_seed(0)
    T = docs[-1]
    cu = torch.tensor(docs, dtype=torch.int32, device=cuda)
    maxlen = max(b - a for a, b in zip(docs, docs[1:]))
    pos = torch.cat([torch.arange(b - a) for a, b in zip(docs, docs[1:])]).to(cuda)
    cos, sin = (t.to(cuda) for t in _tables(maxlen, D))
    qkv = torch.randn(T, (hq + 2 * hkv) * D, device=cuda).bfloat16()
    do = torch.randn(T, hq, D, device=cuda).bfloat16()
    scale = 1 / math.sqrt(D)
    q = qkv[:, : hq * D].view(T, hq, D)
    k = qkv[:, hq * D:(hq + hkv) * D].view(T, hkv, D)
    v = qkv[:, (hq + hkv) * D:].view(T, hkv, D)
    o, lse = ops.flash_attn_fwd(q, k, v, cu, maxlen, scale, causal, window)
    ref = ops.flash_attn_bwd_qkv(do, qkv, hq, hkv, D, o, lse, cu, maxlen, scale, causal, window)
    ops.rope_(ref, cos, sin, pos, hq + hkv, D, True)
    got = ops.flash_attn_bwd_qkv_rope(do, qkv, hq, hkv, D, o, lse, cu, maxlen, scale, causal, cos, sin, pos, window)
    assert torch.equal(got[:, (hq + hkv) * D:], ref[:, (hq + hkv) * D:])  # dV untouched
    for name, sl in (("dq", slice(0, hq * D)), ("dk", slice(hq * D, (hq + hkv) * D))):
        r = _rel(got[:, sl], ref[:, sl])
        assert r < 8e-3, (name, r)  # one bf16 rounding fewer than the two-pass reference


def test_model_grads_fused_vs_separate(cuda, monkeypatch):
    """llama-tiny's gradients with the fused epilogue vs the separate RoPE pass."""
    from dtg.models import build_model, resolve_config
    from dtg.ops import functional as F_

    cfg = resolve_config("llama-tiny-d128")
    out = {}
    for fused in (False, True):
        monkeypatch.setattr(F_, "_FA_ROPE_FUSED", fused)
        torch.manual_seed(0)
        model = build_model(cfg, device=torch.device("cuda"))
        ids = torch.randint(0, cfg.vocab_size, (2, 256), generator=torch.Generator().manual_seed(0)).to(cuda)
        model(input_ids=ids, labels=ids).loss.backward()
        out[fused] = {n: p.grad.float().clone() for n, p in model.named_parameters() if p.grad is not None}
    for n, g in out[False].items():
        assert _rel(out[True][n], g) < 2e-2, n
