"""Pretrained weight loading from HF safetensors directories.

The 405B chapter loads real weights when they are on local disk (`--init-from <dir>` with
`model-*.safetensors`).  Instead of the reference's rank-0 full load + broadcast of 811 GB,
every rank memory-maps the safetensors files and copies only the slices it owns (its FSDP
shard / ZeRO slice / TP shard), converting HF's split q/k/v and gate/up tensors to the fused
layout on the fly.
"""
from __future__ import annotations

import glob
import os

import torch


class _LazyHF:
    def __init__(self, path):
        from safetensors import safe_open

        self.files = {}
        for f in sorted(glob.glob(os.path.join(path, "*.safetensors"))):
            h = safe_open(f, framework="pt")
            for k in h.keys():
                self.files[k] = h

    def get(self, k):
        return self.files[k].get_tensor(k)


def _fused_full(hf: _LazyHF, name: str, cfg):
    """Full (un-TP-sharded) tensor of one of our parameter names."""
    if name.endswith("self_attn.qkv_proj.weight"):
        p = "model." + name[: -len("qkv_proj.weight")]
        return torch.cat([hf.get(p + "q_proj.weight"), hf.get(p + "k_proj.weight"), hf.get(p + "v_proj.weight")], 0)
    if name.endswith("mlp.gate_up_proj.weight"):
        p = "model." + name[: -len("gate_up_proj.weight")]
        return torch.cat([hf.get(p + "gate_proj.weight"), hf.get(p + "up_proj.weight")], 0)
    if name == "lm_head.weight":
        t = hf.get("lm_head.weight")
    else:
        t = hf.get("model." + name)
    if name in ("embed_tokens.weight", "lm_head.weight") and t.shape[0] < cfg.vocab_size:
        # pretrained vocabulary smaller than the config (rime: 128,256 -> 156,939 tokens):
        # resize_token_embeddings semantics, new rows = mean of the pretrained rows
        from . import mean_resized_rows

        t = mean_resized_rows(t, cfg.vocab_size)
    return t


@torch.no_grad()
def load_pretrained(engine, path: str, cfg):
    from ..parallel.tensor_parallel import shard_full_state_dict

    hf = _LazyHF(path)
    tp = getattr(engine.module, "tp", None)
    tp_rank, tp_size = (tp.rank, tp.size) if tp is not None and tp.enabled else (0, 1)
    cache = {}
    for name, start, n, pview, _ in engine.ckpt_pieces():
        if name not in cache:
            full = _fused_full(hf, name, cfg)
            if tp_size > 1:
                full = shard_full_state_dict({name: full}, cfg, tp_rank, tp_size)[name]
            cache = {name: full.reshape(-1)}
        pview.reshape(-1).copy_(cache[name][start:start + n].to(pview.dtype))
    sync = getattr(engine, "sync_params_after_load", None)
    if sync is not None:
        sync()
