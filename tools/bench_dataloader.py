#!/usr/bin/env python3
"""Packed-sequence data-loading throughput (reference 00-rime/packed_dataset.py, SURVEY E8,
BASELINE rows 1-2: 91k tok/s on 1 process, 605k tok/s on 8, with num_workers=8).

The reference collate builds an unused O(T^2) mask per 8192-token sample; this framework's
collator emits position ids + cu_seqlens in O(T).  Prints tokens/s every 50 batches on local
rank 0 and the first batch per rank (duplication check), like the reference.

    python tools/bench_dataloader.py                       # 1 process
    torchrun --standalone --nproc-per-node=8 tools/bench_dataloader.py
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import dtg  # noqa: E402,F401
from dtg.data import PackedCollator, SyntheticPacked, build_dataloader  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, default=1000)
    ap.add_argument("--seq-length", type=int, default=8192)
    ap.add_argument("--batch-size", type=int, default=1)
    ap.add_argument("--num-workers", type=int, default=8)
    ap.add_argument("--eos", type=int, default=128262)
    ap.add_argument("--vocab", type=int, default=156939)
    ap.add_argument("--json", action="store_true")
    a = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
    ds = SyntheticPacked(a.batches * a.batch_size * world + 16, a.seq_length, a.vocab, a.eos, mean_doc_len=600)
    dl = build_dataloader(ds, a.batch_size, PackedCollator(a.eos), dp_size=world, dp_rank=rank, shuffle=False,
                          num_workers=a.num_workers, prefetch_factor=4, pin_memory=False)
    tokens = 0
    t0 = time.time()
    for i, b in enumerate(dl):
        if i == 0:
            print(f"[rank {rank}] first batch ids[:8] = {b['input_ids'][0, :8].tolist()}", flush=True)
        tokens += b["input_ids"].numel()
        if (i + 1) % 50 == 0 and int(os.environ.get("LOCAL_RANK", "0")) == 0:
            print(f"{tokens / (time.time() - t0):.0f} tok/s after {tokens} tokens", flush=True)
        if i + 1 >= a.batches:
            break
    el = time.time() - t0
    t = torch.tensor([tokens], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t)
    if rank == 0:
        rec = {"tokens": int(t.item()), "seconds": el, "tok_per_s_total": t.item() / el, "world": world,
               "num_workers": a.num_workers}
        print(json.dumps(rec) if a.json else f"aggregate {rec['tok_per_s_total']:.0f} tok/s over {world} process(es)")
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
