"""Conversion between this repo's fused-weight layout and HF transformers state dicts.

Used by the parity tests (HF is the numerical oracle) and to import/export
pretrained checkpoints (the 405B chapter loads HF-format weights when they are on disk).
"""
from __future__ import annotations

import torch

from .config import GPT2Config, LlamaConfig


def llama_to_hf(sd: dict, cfg: LlamaConfig) -> dict:
    d = cfg.head_dim
    nq, nkv = cfg.num_attention_heads, cfg.num_key_value_heads
    out = {}
    for k, v in sd.items():
        if k.endswith("self_attn.qkv_proj.weight"):
            pre = k[: -len("qkv_proj.weight")]
            q, kk, vv = v.split([nq * d, nkv * d, nkv * d], dim=0)
            out["model." + pre + "q_proj.weight"] = q
            out["model." + pre + "k_proj.weight"] = kk
            out["model." + pre + "v_proj.weight"] = vv
        elif k.endswith("self_attn.qkv_proj.bias"):
            pre = k[: -len("qkv_proj.bias")]
            q, kk, vv = v.reshape(-1).split([nq * d, nkv * d, nkv * d], dim=0)
            out["model." + pre + "q_proj.bias"] = q
            out["model." + pre + "k_proj.bias"] = kk
            out["model." + pre + "v_proj.bias"] = vv
        elif k.endswith("mlp.gate_up_proj.weight"):
            pre = k[: -len("gate_up_proj.weight")]
            g, u = v.chunk(2, dim=0)
            out["model." + pre + "gate_proj.weight"] = g
            out["model." + pre + "up_proj.weight"] = u
        elif k == "lm_head.weight":
            out[k] = v
        else:
            out["model." + k] = v
    if cfg.tie_word_embeddings:
        out["lm_head.weight"] = out["model.embed_tokens.weight"]
    return out


def llama_from_hf(hf_sd: dict, cfg: LlamaConfig) -> dict:
    out = {}
    L = cfg.num_hidden_layers
    for i in range(L):
        p = f"model.layers.{i}."
        out[f"layers.{i}.self_attn.qkv_proj.weight"] = torch.cat(
            [hf_sd[p + "self_attn.q_proj.weight"], hf_sd[p + "self_attn.k_proj.weight"], hf_sd[p + "self_attn.v_proj.weight"]], 0)
        if p + "self_attn.q_proj.bias" in hf_sd:
            out[f"layers.{i}.self_attn.qkv_proj.bias"] = torch.cat(
                [hf_sd[p + "self_attn.q_proj.bias"], hf_sd[p + "self_attn.k_proj.bias"],
                 hf_sd[p + "self_attn.v_proj.bias"]], 0)[:, None]
        out[f"layers.{i}.self_attn.o_proj.weight"] = hf_sd[p + "self_attn.o_proj.weight"]
        out[f"layers.{i}.mlp.gate_up_proj.weight"] = torch.cat([hf_sd[p + "mlp.gate_proj.weight"], hf_sd[p + "mlp.up_proj.weight"]], 0)
        out[f"layers.{i}.mlp.down_proj.weight"] = hf_sd[p + "mlp.down_proj.weight"]
        out[f"layers.{i}.input_layernorm.weight"] = hf_sd[p + "input_layernorm.weight"]
        out[f"layers.{i}.post_attention_layernorm.weight"] = hf_sd[p + "post_attention_layernorm.weight"]
    out["embed_tokens.weight"] = hf_sd["model.embed_tokens.weight"]
    out["norm.weight"] = hf_sd["model.norm.weight"]
    if not cfg.tie_word_embeddings:
        out["lm_head.weight"] = hf_sd["lm_head.weight"]
    return out


def gpt2_to_hf(sd: dict, cfg: GPT2Config) -> dict:
    out = {}
    ren = {"c_attn": "attn.c_attn", "c_proj": "attn.c_proj", "c_fc": "mlp.c_fc", "mlp_proj": "mlp.c_proj"}
    for k, v in sd.items():
        if k == "wte.weight" or k == "wpe.weight" or k.startswith("ln_f"):
            out["transformer." + k] = v
            continue
        parts = k.split(".")  # h.{i}.{mod}.{weight|bias}
        i, mod, kind = parts[1], parts[2], parts[3]
        if mod in ren:
            name = f"transformer.h.{i}.{ren[mod]}.{kind}"
            out[name] = v.t().contiguous() if kind == "weight" else v
        else:
            out[f"transformer.h.{i}.{mod}.{kind}"] = v
    out["lm_head.weight"] = out["transformer.wte.weight"]
    return out


def hf_llama_config(cfg: LlamaConfig):
    """The transformers config of the same architecture (LlamaConfig / MistralConfig / Qwen2Config)."""
    common = dict(
        vocab_size=cfg.vocab_size, hidden_size=cfg.hidden_size, intermediate_size=cfg.intermediate_size,
        num_hidden_layers=cfg.num_hidden_layers, num_attention_heads=cfg.num_attention_heads,
        num_key_value_heads=cfg.num_key_value_heads, rms_norm_eps=cfg.rms_norm_eps,
        rope_theta=cfg.rope_theta, rope_scaling=cfg.rope_scaling, max_position_embeddings=cfg.max_position_embeddings,
        tie_word_embeddings=cfg.tie_word_embeddings, use_cache=False)
    if cfg.model_type == "qwen2":
        from transformers import Qwen2Config

        return Qwen2Config(use_sliding_window=cfg.sliding_window is not None, sliding_window=cfg.sliding_window, **common)
    if cfg.model_type == "mistral":
        from transformers import MistralConfig

        return MistralConfig(head_dim=cfg.head_dim, sliding_window=cfg.sliding_window, **common)
    from transformers import LlamaConfig as HFLlamaConfig

    return HFLlamaConfig(head_dim=cfg.head_dim, attention_bias=cfg.attention_bias, mlp_bias=False, **common)


def hf_causal_lm_class(cfg: LlamaConfig):
    import transformers

    return {"qwen2": transformers.Qwen2ForCausalLM, "mistral": transformers.MistralForCausalLM}.get(
        cfg.model_type, transformers.LlamaForCausalLM)


def hf_gpt2_config(cfg: GPT2Config):
    from transformers import GPT2Config as HFGPT2Config

    return HFGPT2Config(
        vocab_size=cfg.vocab_size, n_positions=cfg.n_positions, n_embd=cfg.n_embd, n_layer=cfg.n_layer,
        n_head=cfg.n_head, n_inner=cfg.n_inner, activation_function=cfg.activation_function,
        resid_pdrop=0.0, embd_pdrop=0.0, attn_pdrop=0.0, layer_norm_epsilon=cfg.layer_norm_epsilon, use_cache=False,
    )
