"""Tensor / sequence / 2-D parallel setup.

The Llama model implements Megatron-style TP natively (`LlamaForCausalLM(cfg, tp_group=...)`):
column-parallel QKV and gate|up, row-parallel o_proj and down_proj, sequence-parallel norms with
all-gather / reduce-scatter over the token dimension, vocab-parallel embedding and lm_head with a
vocab-parallel fused cross entropy.  This module provides the mesh construction and the mapping
between full (single-device) weights and TP shards, used for initialisation from a full state
dict, checkpoint export and the equivalence tests.

TP ranks of one group are consecutive global ranks, i.e. the GPUs of one xGMI-connected node,
so every TP collective stays on the fully connected intra-node fabric; the dp dimension spans
nodes (reference ch06 mesh (num_nodes, gpus_per_node) / ch07 (world // tp, tp)).
"""
from __future__ import annotations

from typing import Dict

import torch
import torch.distributed as dist


def make_mesh(tp: int):
    """Returns (dp_group, tp_group, dp_rank, tp_rank, dp_size) for a (world//tp, tp) mesh.

    Unlike the reference (07 asserts tp > 1), tp=1 (pure data parallel) and
    tp=world (pure TP) are allowed."""
    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    assert world % tp == 0, f"world size {world} must be divisible by tp={tp}"
    dp = world // tp
    if world == 1:
        return None, None, 0, 0, 1
    tp_group = dp_group = None
    for d in range(dp):
        ranks = list(range(d * tp, (d + 1) * tp))
        g = dist.new_group(ranks)
        if rank in ranks:
            tp_group = g
    for t in range(tp):
        ranks = list(range(t, world, tp))
        g = dist.new_group(ranks)
        if rank in ranks:
            dp_group = g
    return dp_group, tp_group, rank // tp, rank % tp, dp


def _rows(t: torch.Tensor, r: int, n: int) -> torch.Tensor:
    k = t.shape[0] // n
    return t[r * k:(r + 1) * k]


def _cols(t: torch.Tensor, r: int, n: int) -> torch.Tensor:
    k = t.shape[1] // n
    return t[:, r * k:(r + 1) * k]


def shard_full_state_dict(full: Dict[str, torch.Tensor], cfg, tp_rank: int, tp_size: int) -> Dict[str, torch.Tensor]:
    """Full Llama state dict (fused layout) -> this TP rank's shard state dict."""
    d = cfg.head_dim
    nq, nkv = cfg.num_attention_heads, cfg.num_key_value_heads
    out = {}
    for k, v in full.items():
        if k.endswith("self_attn.qkv_proj.weight") or k.endswith("self_attn.qkv_proj.bias"):
            q, kk, vv = v.split([nq * d, nkv * d, nkv * d], 0)
            out[k] = torch.cat([_rows(q, tp_rank, tp_size), _rows(kk, tp_rank, tp_size), _rows(vv, tp_rank, tp_size)], 0)
        elif k.endswith("mlp.gate_up_proj.weight"):
            g, u = v.chunk(2, 0)
            out[k] = torch.cat([_rows(g, tp_rank, tp_size), _rows(u, tp_rank, tp_size)], 0)
        elif k.endswith("self_attn.o_proj.weight") or k.endswith("mlp.down_proj.weight"):
            out[k] = _cols(v, tp_rank, tp_size)
        elif k in ("embed_tokens.weight", "lm_head.weight"):
            out[k] = _rows(v, tp_rank, tp_size)
        else:  # norms: replicated
            out[k] = v
    return out


def unshard_state_dicts(shards, cfg) -> Dict[str, torch.Tensor]:
    """Inverse of shard_full_state_dict over all TP ranks' state dicts (rank order)."""
    d = cfg.head_dim
    n = len(shards)
    nq, nkv = cfg.num_attention_heads // n, cfg.num_key_value_heads // n
    out = {}
    for k in shards[0]:
        parts = [s[k] for s in shards]
        if k.endswith("self_attn.qkv_proj.weight") or k.endswith("self_attn.qkv_proj.bias"):
            qs, ks, vs = zip(*[p.split([nq * d, nkv * d, nkv * d], 0) for p in parts])
            out[k] = torch.cat(list(qs) + list(ks) + list(vs), 0)
        elif k.endswith("mlp.gate_up_proj.weight"):
            gs, us = zip(*[p.chunk(2, 0) for p in parts])
            out[k] = torch.cat(list(gs) + list(us), 0)
        elif k.endswith("self_attn.o_proj.weight") or k.endswith("mlp.down_proj.weight"):
            out[k] = torch.cat(parts, 1)
        elif k in ("embed_tokens.weight", "lm_head.weight"):
            out[k] = torch.cat(parts, 0)
        else:
            out[k] = parts[0]
    return out
