#!/usr/bin/env python3
"""hipBLASLt ceiling check: TN GEMMs at square and Llama shapes, random vs zero operands (DVFS)."""
import torch, json
dev = torch.device("cuda")
def t(fn, it=20):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it): fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / it
for (M, N, K) in [(8192, 8192, 8192), (16384, 16384, 16384), (16384, 28672, 4096), (16384, 4096, 14336), (32768, 28672, 4096)]:
    for init in ("randn", "zeros"):
        a = (torch.randn if init == "randn" else torch.zeros)(M, K, device=dev, dtype=torch.bfloat16)
        b = (torch.randn if init == "randn" else torch.zeros)(N, K, device=dev, dtype=torch.bfloat16)
        ms = t(lambda: torch.mm(a, b.t()))
        print(json.dumps({"M": M, "N": N, "K": K, "init": init, "ms": round(ms, 3), "TF": round(2 * M * N * K / ms / 1e9, 1)}), flush=True)
        del a, b
