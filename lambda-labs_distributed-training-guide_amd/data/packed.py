"""Packed-sequence collation (00-rime) in O(T).

A packed row holds several documents separated by EOS.  Position ids restart at 0 after every
EOS, and attention must stay inside each document.  The reference builds (and discards) a
T x T additive mask per sample and relies on HF's flash-attn varlen path keyed off the
position ids; here the collator emits `cu_seqlens` (int32 document boundaries over the
flattened [B*T] batch) and `max_seqlen` directly, which the varlen flash kernel consumes.

Fixes of the reference's defects: no in-place write of the EOS into the
dataset tensor, a single-EOS row works, no O(T^2) mask.
"""
from __future__ import annotations

from typing import Dict, List, Sequence

import torch


def packed_position_ids(x: torch.Tensor, eos_id: int):
    """Position ids for one packed row (restart after each EOS) and its document lengths.

    The last token is treated as an EOS (the reference forces x[-1] = eos)."""
    T = x.shape[0]
    is_eos = x == eos_id
    is_eos = is_eos.clone()
    is_eos[-1] = True
    ends = torch.nonzero(is_eos).flatten() + 1  # exclusive ends of each document
    starts = torch.cat([ends.new_zeros(1), ends[:-1]])
    lengths = ends - starts
    pos = torch.arange(T) - torch.repeat_interleave(starts, lengths)
    return pos, lengths


class PackedCollator:
    """Collate packed rows -> {input_ids, labels, position_ids, cu_seqlens, max_seqlen, num_valid}."""

    def __init__(self, eos_id: int, force_last_eos: bool = True):
        self.eos_id = eos_id
        self.force_last_eos = force_last_eos

    def __call__(self, samples: Sequence[Dict[str, torch.Tensor]]):
        rows, poss, lens = [], [], []
        for s in samples:
            x = torch.as_tensor(s["input_ids"]).clone()
            if self.force_last_eos:
                x[-1] = self.eos_id
            p, l = packed_position_ids(x, self.eos_id)
            rows.append(x)
            poss.append(p)
            lens.append(l)
        ids = torch.stack(rows)
        lengths = torch.cat(lens)
        cu = torch.zeros(lengths.numel() + 1, dtype=torch.int32)
        cu[1:] = torch.cumsum(lengths, 0)
        labels = ids.clone()  # reference: labels = input_ids after the EOS is forced
        return {
            "input_ids": ids,
            "labels": labels,
            "position_ids": torch.stack(poss),
            "cu_seqlens": cu,
            "max_seqlen": int(lengths.max()),
            "num_valid": int((labels[:, 1:] != -100).sum()),
        }


def dense_collate(samples: List[Dict[str, torch.Tensor]]):
    """default_data_collator equivalent + the host-side `num_valid` count (no device sync)."""
    ids = torch.stack([torch.as_tensor(s["input_ids"]) for s in samples])
    labels = torch.stack([torch.as_tensor(s.get("labels", s["input_ids"])) for s in samples])
    return {"input_ids": ids, "labels": labels, "num_valid": int((labels[:, 1:] != -100).sum())}
