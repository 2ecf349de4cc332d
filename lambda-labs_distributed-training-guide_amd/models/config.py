"""Bundled model configurations.

The GPU boxes have no network, so every model the reference passes via `--model-name`
ships here as JSON.  `resolve_config` accepts the reference's HF hub names
(`meta-llama/Llama-3.1-8B`, `openai-community/gpt2`, ...), the short bundled names
(`llama-3.1-8b`), or a path to an HF-style `config.json`.
"""
from __future__ import annotations

import dataclasses
import json
import os
from typing import Optional

_CFG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "configs")

ALIASES = {
    "openai-community/gpt2": "gpt2",
    "gpt2": "gpt2",
    "meta-llama/llama-2-7b-hf": "llama-2-7b",
    "meta-llama/llama-2-70b-hf": "llama-2-70b",
    "meta-llama/meta-llama-3-8b": "llama-3-8b",
    "meta-llama/llama-3-8b": "llama-3-8b",
    "meta-llama/llama-3.1-8b": "llama-3.1-8b",
    "meta-llama/meta-llama-3.1-8b": "llama-3.1-8b",
    "meta-llama/llama-3.1-8b-instruct": "llama-3.1-8b",
    "meta-llama/meta-llama-3.1-405b": "llama-3.1-405b",
    "meta-llama/llama-3.1-405b": "llama-3.1-405b",
    "meta-llama/llama-3.2-3b-instruct": "llama-3.2-3b",
    "meta-llama/llama-3.2-3b": "llama-3.2-3b",
    "qwen/qwen2.5-0.5b": "qwen2.5-0.5b",
    "qwen/qwen2.5-7b": "qwen2.5-7b",
    "mistralai/mistral-7b-v0.3": "mistral-7b-v0.3",
}


@dataclasses.dataclass
class LlamaConfig:
    vocab_size: int
    hidden_size: int
    intermediate_size: int
    num_hidden_layers: int
    num_attention_heads: int
    num_key_value_heads: int
    head_dim: Optional[int] = None
    rms_norm_eps: float = 1e-5
    rope_theta: float = 10000.0
    rope_scaling: Optional[dict] = None
    max_position_embeddings: int = 4096
    tie_word_embeddings: bool = False
    initializer_range: float = 0.02
    eos_token_id: Optional[int] = None
    hf_name: str = ""
    # llama (Llama-2/3/3.1/3.2), mistral (Llama layout + sliding-window attention), qwen2 (+ q/k/v bias)
    model_type: str = "llama"
    attention_bias: bool = False  # q/k/v projection bias (Qwen2); o_proj never has one here
    sliding_window: Optional[int] = None  # Mistral: keys within this distance (None = full causal)

    def __post_init__(self):
        if self.head_dim is None:
            self.head_dim = self.hidden_size // self.num_attention_heads

    def num_params(self) -> int:
        h, i, v, L = self.hidden_size, self.intermediate_size, self.vocab_size, self.num_hidden_layers
        d = self.head_dim
        attn = h * (self.num_attention_heads + 2 * self.num_key_value_heads) * d + self.num_attention_heads * d * h
        if self.attention_bias:
            attn += (self.num_attention_heads + 2 * self.num_key_value_heads) * d
        layer = attn + 3 * h * i + 2 * h
        return v * h * (1 if self.tie_word_embeddings else 2) + L * layer + h

    def flops_per_token(self, seq_len: int) -> float:
        """Training FLOPs/token: 6 * params (matmuls) + causal attention (fwd 2*2*S/2*d*nh, x3)."""
        n = self.num_params() - self.vocab_size * self.hidden_size * (0 if self.tie_word_embeddings else 1)
        attn = 6 * self.num_hidden_layers * self.num_attention_heads * self.head_dim * seq_len
        return 6 * n + attn


@dataclasses.dataclass
class GPT2Config:
    vocab_size: int = 50257
    n_positions: int = 1024
    n_embd: int = 768
    n_layer: int = 12
    n_head: int = 12
    n_inner: Optional[int] = None
    activation_function: str = "gelu_new"
    resid_pdrop: float = 0.1
    embd_pdrop: float = 0.1
    attn_pdrop: float = 0.1
    layer_norm_epsilon: float = 1e-5
    initializer_range: float = 0.02
    tie_word_embeddings: bool = True
    hf_name: str = ""
    model_type: str = "gpt2"

    @property
    def hidden_size(self):
        return self.n_embd

    @property
    def num_hidden_layers(self):
        return self.n_layer

    @property
    def max_position_embeddings(self):
        return self.n_positions

    def num_params(self) -> int:
        h, L = self.n_embd, self.n_layer
        inner = self.n_inner or 4 * h
        layer = 4 * h + (3 * h * h + 3 * h) + (h * h + h) + (h * inner + inner) + (inner * h + h)
        return self.vocab_size * h + self.n_positions * h + L * layer + 2 * h

    def flops_per_token(self, seq_len: int) -> float:
        return 6 * (self.num_params() - self.n_positions * self.n_embd) + 6 * self.n_layer * self.n_embd * seq_len


LLAMA_FAMILY = ("llama", "mistral", "qwen2")


def _from_dict(d: dict):
    """HF config dict -> our config.  The Llama layout covers llama, mistral and qwen2
    (RMSNorm, RoPE, GQA, SwiGLU); anything else is refused instead of silently mis-built."""
    d = dict(d)
    mt = d.get("model_type", "llama")
    if mt == "gpt2":
        cls = GPT2Config
    elif mt in LLAMA_FAMILY:
        cls = LlamaConfig
        if mt == "qwen2":
            d.setdefault("attention_bias", True)  # Qwen2 always has q/k/v biases
            if not d.get("use_sliding_window", False):
                d["sliding_window"] = None
        if mt == "llama":
            d["sliding_window"] = None
        if d.get("mlp_bias"):
            raise ValueError("mlp_bias=True is not supported (no Llama-family checkpoint uses it)")
    else:
        raise ValueError(f"unsupported model_type {mt!r}; supported: {', '.join(LLAMA_FAMILY)}, gpt2")
    fields = {f.name for f in dataclasses.fields(cls)}
    return cls(**{k: v for k, v in d.items() if k in fields})


def available_configs():
    return sorted(f[:-5] for f in os.listdir(_CFG_DIR) if f.endswith(".json"))


def resolve_config(name: str, **overrides):
    """Config for a bundled name, an HF hub name, or a path to an HF config.json."""
    if os.path.isfile(name):
        with open(name) as fp:
            d = json.load(fp)
    else:
        key = ALIASES.get(name.lower(), name.lower())
        path = os.path.join(_CFG_DIR, key + ".json")
        if not os.path.exists(path):
            raise KeyError(f"unknown model {name!r}; bundled: {available_configs()}")
        with open(path) as fp:
            d = json.load(fp)
    d.update(overrides)
    return _from_dict(d)
