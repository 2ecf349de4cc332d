"""T1: owned models vs HF transformers (installed 5.x) on tiny configs with identical weights."""
import pytest
import math

import torch

import dtg  # noqa: F401
from dtg.models import build_model, count_valid_labels, resolve_config
from dtg.models.hf_compat import (gpt2_to_hf, hf_causal_lm_class, hf_gpt2_config, hf_llama_config, llama_from_hf,
                                  llama_to_hf)


@pytest.mark.parametrize("name", ["llama-tiny", "llama-tiny-d128", "qwen2-tiny", "mistral-tiny"])
def test_llama_matches_hf_loss_logits_grads(name):
    """Llama-family models (Llama, Qwen2 with q/k/v biases, Mistral within its window) against
    the transformers implementation of the same architecture."""
    torch.manual_seed(0)
    cfg = resolve_config(name)
    m = build_model(cfg, device="cpu", dtype=torch.float32)
    if cfg.attention_bias:  # zero-initialised like HF; random here so the bias path is exercised
        with torch.no_grad():
            for n_, p in m.named_parameters():
                if n_.endswith(".bias"):
                    p.normal_(0, 0.1)
    hf = hf_causal_lm_class(cfg)(hf_llama_config(cfg)).float()
    hf.load_state_dict(llama_to_hf(m.state_dict(), cfg), strict=True)
    ids = torch.randint(0, cfg.vocab_size, (2, 40))
    a = m(input_ids=ids, labels=ids, return_logits=True)
    b = hf(input_ids=ids, labels=ids)
    torch.testing.assert_close(a.logits, b.logits, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(a.loss, b.loss, atol=1e-5, rtol=1e-5)
    a.loss.backward()
    b.loss.backward()
    ga = llama_to_hf({n: p.grad for n, p in m.named_parameters()}, cfg)
    for n, p in hf.named_parameters():
        if n == "lm_head.weight" and cfg.tie_word_embeddings:
            continue
        torch.testing.assert_close(ga[n], p.grad, atol=1e-4, rtol=1e-3, msg=n)


def test_unsupported_model_type_is_refused():
    with pytest.raises(ValueError, match="unsupported model_type"):
        resolve_config("llama-tiny", model_type="gemma")


def test_mistral_sliding_window_matches_hf_beyond_window():
    """Rows longer than the window (mistral-tiny: 64) use sliding-window attention, like HF."""
    torch.manual_seed(0)
    cfg = resolve_config("mistral-tiny")
    m = build_model(cfg, device="cpu", dtype=torch.float32)
    hf = hf_causal_lm_class(cfg)(hf_llama_config(cfg)).float()
    hf.load_state_dict(llama_to_hf(m.state_dict(), cfg), strict=True)
    ids = torch.randint(0, cfg.vocab_size, (2, 150))
    a = m(input_ids=ids, labels=ids, return_logits=True)
    b = hf(input_ids=ids, labels=ids)
    torch.testing.assert_close(a.logits, b.logits, atol=1e-4, rtol=1e-4)
    full = resolve_config("mistral-tiny", sliding_window=None)
    m2 = build_model(full, device="cpu", dtype=torch.float32)
    m2.load_state_dict(m.state_dict())
    assert not torch.allclose(m2(input_ids=ids, return_logits=True).logits[:, 100:], a.logits[:, 100:], atol=1e-3)


@pytest.mark.parametrize("name", ["llama-tiny", "qwen2-tiny"])
def test_llama_hf_roundtrip_state_dict(name):
    cfg = resolve_config(name)
    m = build_model(cfg, device="cpu", dtype=torch.float32)
    sd = m.state_dict()
    back = llama_from_hf(llama_to_hf(sd, cfg), cfg)
    assert set(back) == set(sd)
    for k in sd:
        assert torch.equal(back[k], sd[k])


def test_gpt2_matches_hf():
    from transformers import GPT2LMHeadModel as HG

    torch.manual_seed(0)
    cfg = resolve_config("gpt2-tiny")
    g = build_model(cfg, device="cpu", dtype=torch.float32).eval()
    hg = HG(hf_gpt2_config(cfg)).float().eval()
    hg.load_state_dict(gpt2_to_hf(g.state_dict(), cfg), strict=False)
    ids = torch.randint(0, cfg.vocab_size, (2, 33))
    a = g(input_ids=ids, labels=ids, return_logits=True)
    b = hg(input_ids=ids, labels=ids)
    torch.testing.assert_close(a.logits, b.logits, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(a.loss, b.loss, atol=1e-5, rtol=1e-5)


def test_packed_varlen_equals_separate_documents():
    """Packed row with position resets == running each document separately (attention stays
    inside documents, RoPE restarts): the 00-rime varlen path."""
    torch.manual_seed(0)
    cfg = resolve_config("llama-tiny")
    m = build_model(cfg, device="cpu", dtype=torch.float32)
    docs = [torch.randint(0, cfg.vocab_size, (n,)) for n in (7, 12, 5)]
    ids = torch.cat(docs)[None]
    pos = torch.cat([torch.arange(len(d)) for d in docs])[None]
    cu = torch.tensor([0, 7, 19, 24], dtype=torch.int32)
    packed = m(input_ids=ids, position_ids=pos, cu_seqlens=cu, max_seqlen=12, return_logits=True).logits[0]
    sep = torch.cat([m(input_ids=d[None], return_logits=True).logits[0] for d in docs])
    torch.testing.assert_close(packed, sep, atol=1e-4, rtol=1e-4)
    # cu_seqlens derived from position ids when not given
    derived = m(input_ids=ids, position_ids=pos, return_logits=True).logits[0]
    torch.testing.assert_close(derived, packed)


def test_num_valid_hint_matches_internal_count():
    cfg = resolve_config("llama-tiny")
    m = build_model(cfg, device="cpu", dtype=torch.float32)
    ids = torch.randint(0, cfg.vocab_size, (3, 16))
    labels = ids.clone()
    labels[0, 5:] = -100
    a = m(input_ids=ids, labels=labels).loss
    b = m(input_ids=ids, labels=labels, num_valid=count_valid_labels(labels)).loss
    torch.testing.assert_close(a, b)


def test_bundled_configs_param_counts():
    # parameter counts of the reference's models
    expect = {"gpt2": 124.44e6, "llama-2-7b": 6.74e9, "llama-2-70b": 68.98e9, "llama-3-8b": 8.03e9,
              "llama-3.1-405b": 405.85e9, "llama-3.2-3b": 3.21e9,
              # published sizes of the other bundled Llama-layout families
              "qwen2.5-0.5b": 0.494e9, "qwen2.5-7b": 7.62e9, "mistral-7b-v0.3": 7.25e9}
    for name, n in expect.items():
        got = resolve_config(name).num_params()
        assert abs(got - n) / n < 0.01, (name, got)
    assert resolve_config("meta-llama/Llama-3.1-8B").rope_scaling["rope_type"] == "llama3"
    assert resolve_config("openai-community/gpt2").n_layer == 12


@pytest.mark.parametrize("name", ["llama-tiny-d128", "llama-tiny", "gpt2-tiny"])
def test_resize_token_embeddings_mean_rows(name):
    """vocabulary extension keeps old rows, new rows = mean, ties preserved, trains."""
    from dtg.models import build_model, resize_token_embeddings

    torch.manual_seed(0)
    m = build_model(name, device="cpu", dtype=torch.float32)
    old = m.lm_head_weight().detach().clone()
    V = old.shape[0]
    resize_token_embeddings(m, V + 37)
    w = m.lm_head_weight()
    assert w.shape[0] == V + 37 and m.config.vocab_size == V + 37
    assert torch.equal(w[:V], old)
    torch.testing.assert_close(w[V:], old.mean(0, keepdim=True).expand(37, -1))
    if m.config.tie_word_embeddings:
        emb = m.wte.weight if hasattr(m, "wte") else m.embed_tokens.weight
        assert emb is w
    ids = torch.randint(V, V + 37, (2, 16))
    out = m(input_ids=ids, labels=ids)
    out.loss.backward()
    assert torch.isfinite(out.loss)


def test_gpt2_attention_dropout_in_the_flash_op():
    """GPT-2's attention-probability dropout goes through the flash op (the kernels' Philox keep
    mask): p = 0 is the plain op; at p > 0 the output equals the explicit masked softmax with the
    op's own keep mask, the same torch seed reproduces it, and gradients flow."""
    from dtg import ops
    from dtg.ops import _cpu

    torch.manual_seed(0)
    B, S, nh, d = 2, 24, 3, 16
    T = B * S
    qkv = torch.randn(T, 3 * nh * d)
    cu = torch.tensor([0, 10, 30, T], dtype=torch.int32)
    torch.testing.assert_close(ops.attention(qkv, nh, nh, d, cu, 20, dropout_p=1e-9), ops.attention(qkv, nh, nh, d, cu, 20))
    torch.manual_seed(5)
    got = ops.attention(qkv, nh, nh, d, cu, 20, dropout_p=0.25)
    torch.manual_seed(5)
    again = ops.attention(qkv, nh, nh, d, cu, 20, dropout_p=0.25)
    assert torch.equal(got, again)
    torch.manual_seed(5)
    seed, off = _cpu._rng_pair(torch.ops.dtg.philox_rng(qkv, 4))
    q, k, v = qkv.view(T, 3, nh, d).unbind(1)
    _, sc = _cpu.dropout_threshold(0.25)
    want = torch.zeros(T, nh, d)
    for a_, b_ in ((0, 10), (10, 30), (30, T)):
        m = torch.stack([_cpu.dropout_keep(seed, off, h, a_, b_ - a_, b_ - a_, 0.25) for h in range(nh)])
        s = (q[a_:b_].transpose(0, 1) @ k[a_:b_].transpose(0, 1).transpose(1, 2)) / math.sqrt(d)
        s = s.masked_fill(torch.ones(b_ - a_, b_ - a_, dtype=torch.bool).triu(1), float("-inf"))
        want[a_:b_] = ((torch.softmax(s, -1) * m * sc) @ v[a_:b_].transpose(0, 1)).transpose(0, 1)
    torch.testing.assert_close(got, want.reshape(T, nh * d), atol=1e-5, rtol=1e-4)
    frac = torch.cat([_cpu.dropout_keep(seed, off, 0, 0, 256, 256, 0.1).flatten()]).float().mean()
    assert abs(frac - 230 / 256) < 0.01  # keep probability thr / 256
    x = qkv.clone().requires_grad_()
    ops.attention(x, nh, nh, d, cu, 20, dropout_p=0.1).sum().backward()
    assert torch.isfinite(x.grad).all()
