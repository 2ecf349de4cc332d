"""Model zoo: owned Llama-family and GPT-2 causal LMs with bundled configs."""
import torch

from .config import GPT2Config, LlamaConfig, available_configs, resolve_config
from .gpt2 import GPT2LMHeadModel
from .llama import CausalLMOutput, LlamaForCausalLM, count_valid_labels


def build_model(name_or_cfg, device=None, dtype=torch.bfloat16, tp_group=None, init=True, **overrides):
    """Random-init causal LM from a bundled/HF name or a config object (D1: pure bf16 weights)."""
    cfg = resolve_config(name_or_cfg, **overrides) if isinstance(name_or_cfg, str) else name_or_cfg
    if isinstance(cfg, GPT2Config):
        assert tp_group is None, "GPT-2 is the single-GPU/DDP plumbing model; TP is Llama-only"
        m = GPT2LMHeadModel(cfg, device=device, dtype=dtype)
    else:
        m = LlamaForCausalLM(cfg, tp_group=tp_group, device=device, dtype=dtype)
    if init:
        m.init_weights()
    return m


__all__ = ["GPT2Config", "LlamaConfig", "available_configs", "resolve_config", "GPT2LMHeadModel",
           "LlamaForCausalLM", "CausalLMOutput", "count_valid_labels", "build_model"]
