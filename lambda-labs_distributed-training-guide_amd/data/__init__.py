"""Data pipeline: datasets, packed collation, distributed loaders."""
from __future__ import annotations

import os

import torch
from torch.utils.data import DataLoader, DistributedSampler

from .packed import PackedCollator, dense_collate, packed_position_ids
from .synthetic import SyntheticPacked, SyntheticPattern, SyntheticTokens


def build_dataset(name: str, *, tokenizer_name: str = None, seq_length: int = 1024, vocab_size: int = 50257,
                  max_position_embeddings: int = 1024, num_samples: int = 100_000, eos_id: int = None, seed: int = 0):
    """`synthetic` / `synthetic:packed` / `synthetic:packed:<mean_doc_len>` / `synthetic:pattern`
    (learnable progressions, for convergence checks) or an HF dataset name/path.

    Returns (dataset, seq_length, collate_fn)."""
    if name.startswith("synthetic"):
        parts = name.split(":")
        if len(parts) > 1 and parts[1] == "packed":
            mean = int(parts[2]) if len(parts) > 2 else 512
            eos = eos_id if eos_id is not None else vocab_size - 1
            return SyntheticPacked(num_samples, seq_length, vocab_size, eos, mean, seed), seq_length, PackedCollator(eos)
        if len(parts) > 1 and parts[1] == "pattern":
            return SyntheticPattern(num_samples, seq_length, vocab_size, seed=seed), seq_length, dense_collate
        return SyntheticTokens(num_samples, seq_length, vocab_size, seed), seq_length, dense_collate
    if name.startswith("disk:"):
        import datasets

        ds = datasets.Dataset.load_from_disk(name[5:]).with_format("torch")
        eos = eos_id
        return ds, seq_length, (PackedCollator(eos) if eos is not None else dense_collate)
    from .text import load_and_preprocess

    ds, seq_length = load_and_preprocess(name, tokenizer_name, seq_length, max_position_embeddings)
    return ds, seq_length, dense_collate


def seed_worker(worker_id):
    """Deterministic DataLoader workers (related-topics/determinism, E9)."""
    import random

    import numpy as np

    s = torch.initial_seed() % 2**32
    np.random.seed(s)
    random.seed(s)


class ResumableSampler(torch.utils.data.Sampler):
    """Epoch-seeded sharded order (DistributedSampler semantics, also for one rank) that can
    start part-way through an epoch: `skip` samples of this rank's order are not yielded, so a
    resumed run continues the same data order without loading and collating the consumed
    batches (the reference re-reads them)."""

    def __init__(self, dataset, num_replicas: int = 1, rank: int = 0, shuffle: bool = True, drop_last: bool = True,
                 seed: int = 0):
        self.base = DistributedSampler(dataset, num_replicas=num_replicas, rank=rank, shuffle=shuffle,
                                       drop_last=drop_last, seed=seed)
        self.skip = 0

    def set_epoch(self, epoch: int, skip: int = 0):
        self.base.set_epoch(epoch)
        self.skip = skip

    def full_len(self) -> int:
        return len(self.base)

    def __len__(self):
        return max(0, len(self.base) - self.skip)

    def __iter__(self):
        it = iter(self.base)
        for _ in range(self.skip):
            next(it, None)
        return it


def build_dataloader(dataset, batch_size: int, collate_fn, *, dp_size: int = 1, dp_rank: int = 0, shuffle: bool = True,
                     drop_last: bool = True, num_workers: int = 1, prefetch_factor: int = 2, seed: int = 0,
                     pin_memory: bool = True):
    sampler = ResumableSampler(dataset, num_replicas=dp_size, rank=dp_rank, shuffle=shuffle, drop_last=drop_last,
                               seed=seed)
    g = torch.Generator()
    g.manual_seed(seed)
    kw = {}
    if num_workers > 0:
        # GPU runs start workers with "spawn": forking a process that holds a HIP context and
        # tens of GB of pinned host memory (FSDP CPU offload) stalled the parent's first device
        # synchronize indefinitely on MI355X boxes (chapter 05 with --num-workers 2; fine with
        # spawn or 0 workers).  Persistent workers pay the interpreter start-up once per run.
        ctx = os.environ.get("DTG_LOADER_CTX") or ("spawn" if torch.cuda.is_available() else None)
        kw = dict(prefetch_factor=prefetch_factor, worker_init_fn=seed_worker, persistent_workers=ctx == "spawn")
        if ctx:
            kw["multiprocessing_context"] = ctx
    pin = pin_memory and torch.cuda.is_available() and os.environ.get("DTG_LOADER_PIN", "1") == "1"
    return DataLoader(dataset, batch_size=batch_size, sampler=sampler, drop_last=drop_last, collate_fn=collate_fn,
                      num_workers=num_workers, generator=g, pin_memory=pin, **kw)


__all__ = ["ResumableSampler", "PackedCollator", "dense_collate", "packed_position_ids", "SyntheticPacked", "SyntheticTokens",
           "build_dataset", "build_dataloader", "seed_worker"]
