"""Synthetic datasets (the GPU boxes have no network).

`SyntheticTokens`: fixed-length rows of uniform random token ids, deterministic per index.
`SyntheticPacked`: 00-rime-style packed rows -- random documents (geometric lengths) joined
with EOS, deterministic per index.  Both are map-style datasets, so DistributedSampler,
resume skip-ahead and the loader benchmark work exactly as with a real `datasets.Dataset`.
"""
from __future__ import annotations

import torch
from torch.utils.data import Dataset


class SyntheticTokens(Dataset):
    def __init__(self, num_samples: int, seq_length: int, vocab_size: int, seed: int = 0):
        self.n, self.s, self.v, self.seed = num_samples, seq_length, vocab_size, seed

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        g = torch.Generator().manual_seed(self.seed * 1_000_003 + int(i))
        x = torch.randint(0, self.v, (self.s,), generator=g)
        return {"input_ids": x, "labels": x}


class SyntheticPacked(Dataset):
    def __init__(self, num_samples: int, seq_length: int, vocab_size: int, eos_id: int,
                 mean_doc_len: int = 512, seed: int = 0):
        self.n, self.s, self.v, self.eos, self.mean, self.seed = num_samples, seq_length, vocab_size, eos_id, mean_doc_len, seed

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        g = torch.Generator().manual_seed(self.seed * 1_000_003 + int(i))
        x = torch.randint(0, self.v, (self.s,), generator=g)
        x[x == self.eos] = (self.eos + 1) % self.v
        # document boundaries: geometric gaps with the requested mean length
        p = 1.0 / max(2, self.mean)
        marks = torch.rand(self.s, generator=g) < p
        x[marks] = self.eos
        return {"input_ids": x, "labels": x}
