"""Model zoo: owned Llama-family and GPT-2 causal LMs with bundled configs."""
import torch

from .config import GPT2Config, LlamaConfig, available_configs, resolve_config
from .gpt2 import GPT2LMHeadModel
from .llama import CausalLMOutput, LlamaForCausalLM, count_valid_labels


def build_model(name_or_cfg, device=None, dtype=torch.bfloat16, tp_group=None, init=True, cp_group=None, sp_group=None,
                **overrides):
    """Random-init causal LM from a bundled/HF name or a config object (D1: pure bf16 weights)."""
    cfg = resolve_config(name_or_cfg, **overrides) if isinstance(name_or_cfg, str) else name_or_cfg
    if isinstance(cfg, GPT2Config):
        assert tp_group is None and cp_group is None and sp_group is None, "GPT-2 is the single-GPU/DDP plumbing model; TP is Llama-only"
        m = GPT2LMHeadModel(cfg, device=device, dtype=dtype)
    else:
        m = LlamaForCausalLM(cfg, tp_group=tp_group, device=device, dtype=dtype, cp_group=cp_group, sp_group=sp_group)
    if init:
        m.init_weights()
    return m


def mean_resized_rows(w: torch.Tensor, n_rows: int) -> torch.Tensor:
    """[V, H] -> [n_rows, H]: existing rows kept, new rows = mean of the old ones.

    transformers' `resize_token_embeddings(mean_resizing=True)` samples new rows from
    N(mean, 1e-9 * cov) of the old embeddings, i.e. the mean up to ~1e-5 noise; the
    deterministic mean is used here (reference 00-rime/train_llm_01-single-gpu.py:62-66)."""
    if n_rows <= w.shape[0]:
        return w[:n_rows]
    mean = w.float().mean(0, keepdim=True).to(w.dtype)
    return torch.cat([w, mean.expand(n_rows - w.shape[0], -1)], 0)


@torch.no_grad()
def resize_token_embeddings(model, new_vocab: int):
    """HF-style vocabulary resize of an un-wrapped, non-TP model; call it before
    handing the model to a parallel engine.  Tied embeddings stay tied."""
    import torch.nn as nn

    if isinstance(model, GPT2LMHeadModel):
        holders = [(model, "wte")]
        model.config.vocab_size = new_vocab
    else:
        assert not model.tp.enabled, "resize the full model before tensor-parallel sharding"
        holders = [(model, "embed_tokens")] + ([] if model.lm_head is None else [(model, "lm_head")])
        model.config.vocab_size = new_vocab
        model.vocab_local = new_vocab
    for owner, attr in holders:
        mod = getattr(owner, attr)
        old = mod.weight
        new = nn.Parameter(mean_resized_rows(old.data, new_vocab).clone(), requires_grad=old.requires_grad)
        for a in ("_dtg_uses", "_dtg_sequence_parallel"):
            if hasattr(old, a):
                setattr(new, a, getattr(old, a))
        mod.weight = new
    return model


__all__ = ["GPT2Config", "LlamaConfig", "available_configs", "resolve_config", "GPT2LMHeadModel",
           "LlamaForCausalLM", "CausalLMOutput", "count_valid_labels", "build_model", "resize_token_embeddings",
           "mean_resized_rows"]
