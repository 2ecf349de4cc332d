"""Pretrained weight loading from HF safetensors directories.

The 405B chapter loads real weights when they are on local disk (`--init-from <dir>` with
`model-*.safetensors`).  Instead of the reference's rank-0 full load + broadcast of 811 GB
(/root/reference/05-training-llama-405b/train_llm.py: `sync_module_states=True` after a rank-0
`from_pretrained`), every rank memory-maps the safetensors files and reads ONLY the rows of the
slices it owns (its FSDP shard / ZeRO slice / TP shard / pipeline stage): each owned flat range
maps to a row range of our parameter, which maps to row (or, for row-parallel TP weights,
column) ranges of one or more HF tensors, read through `safe_open(...).get_slice`.  HF's split
q/k/v and gate/up tensors are fused on the fly; across the ranks of a job each weight byte is
read from disk once (plus partial rows at slice edges), instead of once per rank.
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
        if not self.files:
            raise FileNotFoundError(f"no *.safetensors under {path}")

    def get(self, k):
        return self.files[k].get_tensor(k)

    def shape(self, k):
        return tuple(self.files[k].get_slice(k).get_shape())

    def rows(self, k, r0, r1, c0=None, c1=None):
        """Rows [r0, r1) (and columns [c0, c1) if given) of tensor k, reading only those bytes."""
        s = self.files[k].get_slice(k)
        if len(s.get_shape()) == 1:
            return s[r0:r1]
        return s[r0:r1] if c0 is None else s[r0:r1, c0:c1]


def _segments(name: str, cfg, tp_rank: int, tp_size: int):
    """Our (TP-local, fused) parameter as a stack of row segments of HF tensors:
    [(hf_name, local_rows, hf_row_offset, (c0, c1) or None)]."""
    d = cfg.head_dim
    if name.endswith("self_attn.qkv_proj.weight") or name.endswith("self_attn.qkv_proj.bias"):
        suf = name.rsplit(".", 1)[1]  # weight | bias
        p = "model." + name[: -len("qkv_proj." + suf)]
        nq, nkv = cfg.num_attention_heads * d // tp_size, cfg.num_key_value_heads * d // tp_size
        return [(p + "q_proj." + suf, nq, tp_rank * nq, None), (p + "k_proj." + suf, nkv, tp_rank * nkv, None),
                (p + "v_proj." + suf, nkv, tp_rank * nkv, None)]
    if name.endswith("mlp.gate_up_proj.weight"):
        p = "model." + name[: -len("gate_up_proj.weight")]
        i = cfg.intermediate_size // tp_size
        return [(p + "gate_proj.weight", i, tp_rank * i, None), (p + "up_proj.weight", i, tp_rank * i, None)]
    if name.endswith("self_attn.o_proj.weight") or name.endswith("mlp.down_proj.weight"):
        cols = (cfg.num_attention_heads * d if "o_proj" in name else cfg.intermediate_size) // tp_size
        return [("model." + name, cfg.hidden_size, 0, (tp_rank * cols, (tp_rank + 1) * cols))]
    if name in ("embed_tokens.weight", "lm_head.weight"):
        v = cfg.vocab_size // tp_size
        return [("lm_head.weight" if name == "lm_head.weight" else "model." + name, v, tp_rank * v, None)]
    return [("model." + name, None, 0, None)]  # norms: replicated, 1-D


def _read_rows(hf: _LazyHF, name: str, r0: int, r1: int, cfg, tp_rank: int, tp_size: int):
    """Rows [r0, r1) of our TP-local parameter `name`."""
    parts, base = [], 0
    for hk, nrows, off, cols in _segments(name, cfg, tp_rank, tp_size):
        if nrows is None:
            return hf.rows(hk, r0, r1)
        lo, hi = max(r0, base), min(r1, base + nrows)
        if lo < hi:
            a, b = cols if cols is not None else (None, None)
            parts.append(hf.rows(hk, off + lo - base, off + hi - base, a, b))
        base += nrows
    return torch.cat(parts, 0) if len(parts) > 1 else parts[0]


def _vocab_resized(hf: _LazyHF, name: str, cfg) -> bool:
    if name not in ("embed_tokens.weight", "lm_head.weight"):
        return False
    k = "lm_head.weight" if name == "lm_head.weight" else "model." + name
    return hf.shape(k)[0] < cfg.vocab_size


def _fused_full(hf: _LazyHF, name: str, cfg):
    """Full (un-TP-sharded) tensor of an embedding whose pretrained vocabulary is smaller than
    the config's (rime: 128,256 -> 156,939 tokens): resize_token_embeddings semantics, new rows =
    mean of the pretrained rows."""
    from . import mean_resized_rows

    t = hf.get("lm_head.weight" if name == "lm_head.weight" else "model." + name)
    return mean_resized_rows(t, cfg.vocab_size)


def _global_name(engine):
    from ..train.checkpoint import _name_map

    return _name_map(engine)


@torch.no_grad()
def load_pretrained(engine, path: str, cfg):
    """Copy this rank's owned slices of every parameter from an HF safetensors directory."""
    from ..parallel.tensor_parallel import shard_full_state_dict

    hf = _LazyHF(path)
    tp = getattr(engine.module, "tp", None)
    tp_rank, tp_size = (tp.rank, tp.size) if tp is not None and tp.enabled else (0, 1)
    gname = _global_name(engine)
    resized = {}
    for name, start, n, pview, _ in engine.ckpt_pieces():
        g = gname(name)
        if g == "lm_head.weight" and cfg.tie_word_embeddings:
            g = "embed_tokens.weight"
        if _vocab_resized(hf, g, cfg):
            if g not in resized:
                full = _fused_full(hf, g, cfg)
                if tp_size > 1:
                    full = shard_full_state_dict({g: full}, cfg, tp_rank, tp_size)[g]
                resized = {g: full.reshape(-1)}
            pview.reshape(-1).copy_(resized[g][start:start + n].to(pview.dtype))
            continue
        cols = _row_width(g, cfg, tp_size)
        if cols is None:  # 1-D
            src = _read_rows(hf, g, start, start + n, cfg, tp_rank, tp_size)
            pview.reshape(-1).copy_(src.reshape(-1).to(pview.dtype))
            continue
        r0, r1 = start // cols, -(-(start + n) // cols)
        rows = _read_rows(hf, g, r0, r1, cfg, tp_rank, tp_size).reshape(-1)
        o = start - r0 * cols
        pview.reshape(-1).copy_(rows[o:o + n].to(pview.dtype))
    sync = getattr(engine, "sync_params_after_load", None)
    if sync is not None:
        sync()


def _row_width(name: str, cfg, tp_size: int):
    """Columns of our TP-local parameter (None for 1-D)."""
    if name.endswith("layernorm.weight") or name == "norm.weight":
        return None
    if name.endswith("qkv_proj.bias"):
        return 1  # stored as a [rows, 1] column
    if name.endswith("self_attn.o_proj.weight"):
        return cfg.num_attention_heads * cfg.head_dim // tp_size
    if name.endswith("mlp.down_proj.weight"):
        return cfg.intermediate_size // tp_size
    return cfg.hidden_size
