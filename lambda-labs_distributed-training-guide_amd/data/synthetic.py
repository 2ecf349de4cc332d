"""Synthetic datasets (the GPU boxes have no network).

`SyntheticTokens`: fixed-length rows of uniform random token ids, deterministic per index.
`SyntheticPacked`: 00-rime-style packed rows -- random documents (geometric lengths) joined
with EOS, deterministic per index.
`SyntheticPattern`: LEARNABLE rows -- arithmetic progressions x_t = (start + stride * t) mod V
with a random start and a stride drawn from a few values, so the next token follows from the
previous two (the stride is read off the context through attention).  A correct training stack
drives the loss from ln V towards 0 on it; uniform random tokens (the benchmark data) pin it at
ln V whatever the stack does.  Both are map-style datasets, so DistributedSampler,
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


class SyntheticPattern(Dataset):
    def __init__(self, num_samples: int, seq_length: int, vocab_size: int, strides=(1, 2, 3, 5, 7),
                 seed: int = 0):
        self.n, self.s, self.v, self.strides, self.seed = num_samples, seq_length, vocab_size, tuple(strides), seed

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        g = torch.Generator().manual_seed(self.seed * 1_000_003 + int(i))
        start = int(torch.randint(0, self.v, (1,), generator=g))
        k = self.strides[int(torch.randint(0, len(self.strides), (1,), generator=g))]
        x = (start + k * torch.arange(self.s)) % self.v
        return {"input_ids": x, "labels": x}
