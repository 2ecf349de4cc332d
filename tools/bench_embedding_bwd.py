#!/usr/bin/env python3
"""Embedding-backward (dtg::embedding_bwd_) timing at the 8B shapes: TP 1, TP 8 (7/8 of the ids
out of shard, -1), and one token covering 3/4 of the batch (profiles/r2/s39/emb_bench.jsonl)."""
import json
import os
import sys
import time

import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import dtg, dtg.ops
d = torch.ops.dtg
dev = torch.device("cuda:0")
for name, T, V, H, skip in [("tp1_8b", 16384, 128256, 4096, 0.0), ("tp8_8b", 16384, 16032, 4096, 7/8), ("one_hot_run", 16384, 128256, 4096, -1)]:
    ids = torch.randint(0, V, (T,), device=dev)
    if skip > 0: ids[torch.rand(T, device=dev) < skip] = -1
    if skip < 0: ids[: T * 3 // 4] = 13  # one token covering 3/4 of the batch
    dy = torch.randn(T, H, device=dev).bfloat16()
    out = torch.zeros(V, H, device=dev).bfloat16()
    for _ in range(3): d.embedding_bwd_(out, ids, dy)
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(20): d.embedding_bwd_(out, ids, dy)
    torch.cuda.synchronize()
    print(json.dumps({"case": name, "T": T, "V": V, "H": H, "us": round((time.perf_counter() - t) / 20 * 1e6, 1)}), flush=True)
