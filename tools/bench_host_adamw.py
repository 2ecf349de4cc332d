#!/usr/bin/env python3
"""Host AdamW (FSDP CPU offload) throughput per ISA path: python tools/bench_host_adamw.py"""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import os, time, torch, dtg, dtg.ops
n = 200_000_000
p = torch.randn(n).bfloat16(); g = torch.randn(n).bfloat16(); m = torch.zeros(n).bfloat16(); v = torch.zeros(n).bfloat16()
for isa in ["scalar", "avx2", "avx512"]:
    os.environ["DTG_HOST_ADAMW_ISA"] = isa
    torch.ops.dtg.adamw_cpu_(p, g, m, v, 1e-3, .9, .999, 1e-8, .01, 1, 1.0)
    t = time.perf_counter()
    for _ in range(3): torch.ops.dtg.adamw_cpu_(p, g, m, v, 1e-3, .9, .999, 1e-8, .01, 2, 1.0)
    dt = (time.perf_counter() - t) / 3
    print(isa, f"{dt*1e3:.1f} ms", f"{14*n/dt/1e9:.1f} GB/s", flush=True)
