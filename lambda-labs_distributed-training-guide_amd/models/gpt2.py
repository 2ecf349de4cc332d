"""GPT-2 causal LM: the default `--model-name openai-community/gpt2` of chapters 01-04.

Semantics match HF GPT2LMHeadModel: learned positions, pre-LayerNorm blocks,
fused QKV projection with bias, GELU-tanh MLP, dropout 0.1, tied lm_head.  Attention uses
the same varlen flash kernel as Llama (head_dim 64); LayerNorm/GELU/dropout are ATen ops
(GPT-2 is the plumbing model, the hot-path kernels target the Llama family).  Linear weights
are stored [out, in] (HF's Conv1D stores [in, out]; `hf_compat` transposes).
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops
from .config import GPT2Config
from .llama import CausalLMOutput, Weight


class _LN(nn.Module):
    def __init__(self, n, eps, device, dtype):
        super().__init__()
        self.eps = eps
        self.weight = nn.Parameter(torch.empty(n, device=device, dtype=dtype))
        self.bias = nn.Parameter(torch.empty(n, device=device, dtype=dtype))

    def forward(self, x):
        return F.layer_norm(x, (x.shape[-1],), self.weight, self.bias, self.eps)


class _Lin(nn.Module):
    def __init__(self, n_in, n_out, device, dtype):
        super().__init__()
        self.weight = nn.Parameter(torch.empty(n_out, n_in, device=device, dtype=dtype))
        self.bias = nn.Parameter(torch.empty(n_out, device=device, dtype=dtype))

    def forward(self, x):
        return ops.linear(x, self.weight, self.bias)


class GPT2Block(nn.Module):
    def __init__(self, cfg: GPT2Config, device=None, dtype=torch.bfloat16):
        super().__init__()
        h = cfg.n_embd
        inner = cfg.n_inner or 4 * h
        self.nh = cfg.n_head
        self.d = h // cfg.n_head
        self.cfg = cfg
        self.ln_1 = _LN(h, cfg.layer_norm_epsilon, device, dtype)
        self.c_attn = _Lin(h, 3 * h, device, dtype)
        self.c_proj = _Lin(h, h, device, dtype)
        self.ln_2 = _LN(h, cfg.layer_norm_epsilon, device, dtype)
        self.c_fc = _Lin(h, inner, device, dtype)
        self.mlp_proj = _Lin(inner, h, device, dtype)

    def forward(self, x, cu, max_seqlen, dense=None):
        p_attn = self.cfg.attn_pdrop if self.training else 0.0
        p_res = self.cfg.resid_pdrop if self.training else 0.0
        qkv = self.c_attn(self.ln_1(x))
        # attention-probability dropout (attn_pdrop, 0.1 in training) runs inside the flash
        # kernels: Philox keep mask drawn in the forward, regenerated in the backward
        a = ops.attention(qkv, self.nh, self.nh, self.d, cu, max_seqlen, dropout_p=p_attn)
        x = x + F.dropout(self.c_proj(a), p_res, self.training)
        m = self.mlp_proj(F.gelu(self.c_fc(self.ln_2(x)), approximate="tanh"))
        return x + F.dropout(m, p_res, self.training)


class GPT2LMHeadModel(nn.Module):
    def __init__(self, cfg: GPT2Config, device=None, dtype=torch.bfloat16):
        super().__init__()
        self.config = cfg
        h = cfg.n_embd
        self.wte = Weight(cfg.vocab_size, h, device=device, dtype=dtype)
        self.wte.weight._dtg_uses = 2  # tied: embedding + lm_head gradient contributions
        self.wpe = Weight(cfg.n_positions, h, device=device, dtype=dtype)
        self.h = nn.ModuleList([GPT2Block(cfg, device, dtype) for _ in range(cfg.n_layer)])
        self.ln_f = _LN(h, cfg.layer_norm_epsilon, device, dtype)
        self._dense_cache = {}

    @property
    def layers(self):
        return self.h

    @torch.no_grad()
    def init_param(self, name: str, p: torch.Tensor):
        """HF GPT-2 init: normal(0, 0.02), residual projections scaled by 1/sqrt(2 n_layer)."""
        std = self.config.initializer_range
        if ".ln_" in name or name.startswith("ln_f"):
            p.fill_(1.0 if name.endswith("weight") else 0.0)
        elif name.endswith("bias"):
            p.zero_()
        elif name.endswith("c_proj.weight") or name.endswith("mlp_proj.weight"):
            p.normal_(0.0, std / math.sqrt(2 * self.config.n_layer))
        else:
            p.normal_(0.0, std)

    @torch.no_grad()
    def init_weights(self):
        for name, p in self.named_parameters():
            if p.device.type != "meta":
                self.init_param(name, p)

    def lm_head_weight(self):
        return self.wte.weight

    def forward(self, input_ids, labels=None, position_ids=None, cu_seqlens=None, max_seqlen=None,
                num_valid=None, return_logits=False, attention_mask=None):
        B, S = input_ids.shape
        T = B * S
        dev = input_ids.device
        ids = input_ids.reshape(-1)
        if position_ids is None:
            key = (B, S, str(dev))
            if key not in self._dense_cache:
                self._dense_cache = {key: (torch.arange(S, device=dev).repeat(B),
                                           torch.arange(0, (B + 1) * S, S, device=dev, dtype=torch.int32))}
            pos, cu = self._dense_cache[key]
            max_seqlen = S
            dense = (B, S)
        else:
            dense = None
            pos = position_ids.reshape(-1).to(torch.long)
            if cu_seqlens is None:
                starts = torch.unique(torch.cat([torch.nonzero(pos == 0).flatten(), torch.arange(0, T, S, device=dev)]))
                cu = torch.cat([starts, torch.tensor([T], device=dev)]).to(torch.int32)
            else:
                cu = cu_seqlens.to(device=dev, dtype=torch.int32)
            if max_seqlen is None:
                max_seqlen = int((cu[1:] - cu[:-1]).max().item())
        x = ops.embedding(ids, self.wte.weight) + F.embedding(pos, self.wpe.weight)
        x = F.dropout(x, self.config.embd_pdrop if self.training else 0.0, self.training)
        for blk in self.h:
            x = blk(x, cu, int(max_seqlen), dense)
        h = self.ln_f(x)
        out = CausalLMOutput()
        if labels is not None:
            shifted = torch.full_like(labels, -100)
            shifted[:, :-1] = labels[:, 1:]
            shifted = shifted.reshape(-1)
            if num_valid is None:
                num_valid = int((shifted != -100).sum().item())
            out.loss = ops.fused_linear_cross_entropy(h, self.wte.weight, shifted, num_valid=num_valid)
        if return_logits or labels is None:
            out.logits = ops.linear(h, self.wte.weight).view(B, S, -1)
        return out
