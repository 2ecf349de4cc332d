#!/usr/bin/env python3
"""Flash-attention kernel micro-benchmark (fwd / bwd) at the model shapes, random data.

    python tools/bench_attention.py --shape llama8b      # B16 S1024 Hq32 Hkv8 D128 causal
    python tools/bench_attention.py --shape rime         # 1 x 8192 packed docs, Hq24 Hkv8
"""
import argparse
import json
import math
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

import dtg  # noqa: E402,F401
import dtg.ops  # noqa: E402,F401

SHAPES = {
    "llama8b": dict(B=16, S=1024, hq=32, hkv=8, d=128, docs=None),
    "llama8b-tp8": dict(B=16, S=1024, hq=4, hkv=1, d=128, docs=None),
    "rime": dict(B=1, S=8192, hq=24, hkv=8, d=128, docs=600),
    "gpt2": dict(B=16, S=1024, hq=12, hkv=12, d=64, docs=None),
    "long": dict(B=2, S=8192, hq=32, hkv=8, d=128, docs=None),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="llama8b", choices=list(SHAPES))
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--sweep", action="store_true",
                    help="constant 16k tokens, S = 512..8192, causal and non-causal (Hq32/Hkv8/D128)")
    ap.add_argument("--ab-bwd", default=None,
                    help="KNOB=v1,v2 with KNOB kv_split or kv_qb (dtg.ops.fa_tuning): backward timed under "
                         "each value in interleaved rounds in ONE process (same device, same clocks), medians "
                         "reported, outputs compared bitwise")
    ap.add_argument("--ab-tolerant", action="store_true",
                    help="--ab-bwd variants that change the summation order: compare within 1e-2 relative")
    a = ap.parse_args()
    if a.ab_bwd:
        var, vals = a.ab_bwd.split("=", 1)
        return ab_bwd(a, var, vals.split(","))
    if a.sweep:
        for S in (512, 1024, 2048, 4096, 8192):
            for causal in (True, False):
                run(a, dict(B=16384 // S, S=S, hq=32, hkv=8, d=128, docs=None), f"sweep_S{S}", causal)
        return
    run(a, SHAPES[a.shape], a.shape, True)


def _inputs(c, causal):
    dev = torch.device("cuda:0")
    B, S, hq, hkv, d = c["B"], c["S"], c["hq"], c["hkv"], c["d"]
    T = B * S
    if c["docs"]:
        g = torch.Generator().manual_seed(0)
        lens, left = [], T
        while left > 0:
            n = min(left, int(torch.randint(64, 2 * c["docs"], (1,), generator=g)))
            lens.append(n)
            left -= n
        cu = torch.tensor([0] + torch.tensor(lens).cumsum(0).tolist(), dtype=torch.int32)
        flops = sum(l * l / (2 if causal else 1) for l in lens) * 4 * d * hq
    else:
        cu = torch.arange(0, T + 1, S, dtype=torch.int32)
        flops = B * S * S / (2 if causal else 1) * 4 * d * hq
    cu = cu.to(dev)
    maxlen = int((cu[1:] - cu[:-1]).max())
    qkv = torch.randn(T, (hq + 2 * hkv) * d, device=dev).bfloat16()
    q = qkv[:, : hq * d].view(T, hq, d)
    k = qkv[:, hq * d:(hq + hkv) * d].view(T, hkv, d)
    v = qkv[:, (hq + hkv) * d:].view(T, hkv, d)
    return q, k, v, cu, maxlen, flops, 1 / math.sqrt(d)


def ab_bwd(a, var, variants, rounds=7):
    import statistics

    cases = [("S1024c", dict(B=16, S=1024, hq=32, hkv=8, d=128, docs=None), True),
             ("S1024c-tp8", SHAPES["llama8b-tp8"], True), ("S1024c-tp4", dict(B=16, S=1024, hq=8, hkv=2, d=128, docs=None), True),
             ("S4096c", dict(B=4, S=4096, hq=32, hkv=8, d=128, docs=None), True),
             ("S8192nc", dict(B=2, S=8192, hq=32, hkv=8, d=128, docs=None), False),
             ("rime", SHAPES["rime"], True)]
    ops = torch.ops.dtg
    for name, c, causal in cases:
        q, k, v, cu, maxlen, flops, scale = _inputs(c, causal)
        qkv = q.as_strided((q.shape[0], q.stride(0)), (q.stride(0), 1))  # the fused projection output
        hq, hkv, d = c["hq"], c["hkv"], c["d"]
        do = torch.randn(q.shape[0], hq, d, device=q.device).bfloat16()
        o, lse = ops.flash_attn_fwd(q, k, v, cu, maxlen, scale, causal)
        ref = None
        times = {vv: [] for vv in variants}
        for r in range(rounds):
            for vv in variants:
                with dtg.ops.fa_tuning(q.device, **{var: int(vv)}):
                    for _ in range(3):
                        g = ops.flash_attn_bwd_qkv(do, qkv, hq, hkv, d, o, lse, cu, maxlen, scale, causal)
                    if ref is None:
                        ref = g.clone()
                    elif r == 0 and not a.ab_tolerant:
                        assert torch.equal(g, ref), (name, vv, (g.float() - ref.float()).abs().max().item())
                    elif r == 0:
                        err = ((g.float() - ref.float()).norm() / ref.float().norm().clamp_min(1e-12)).item()
                        assert err < 1e-2, (name, vv, err)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(a.iters):
                        ops.flash_attn_bwd_qkv(do, qkv, hq, hkv, d, o, lse, cu, maxlen, scale, causal)
                    e1.record()
                    torch.cuda.synchronize()
                    times[vv].append(e0.elapsed_time(e1) / a.iters)
        rec = {"case": name, "bitwise_equal": not a.ab_tolerant}
        for vv in variants:
            med = statistics.median(times[vv])
            rec[vv] = {"ms": round(med, 4), "min_ms": round(min(times[vv]), 4), "TFLOPs": round(2.5 * flops / med / 1e9, 1)}
        print(json.dumps(rec), flush=True)


def run(a, c, name, causal):
    dev = torch.device("cuda:0")
    B, S, hq, hkv, d = c["B"], c["S"], c["hq"], c["hkv"], c["d"]
    T = B * S
    if c["docs"]:
        g = torch.Generator().manual_seed(0)
        lens = []
        left = T
        while left > 0:
            n = min(left, int(torch.randint(64, 2 * c["docs"], (1,), generator=g)))
            lens.append(n)
            left -= n
        cu = torch.tensor([0] + torch.tensor(lens).cumsum(0).tolist(), dtype=torch.int32)
        causal_flops = sum(l * l / 2 for l in lens) * 4 * d * hq
    else:
        cu = torch.arange(0, T + 1, S, dtype=torch.int32)
        causal_flops = B * S * S / (2 if causal else 1) * 4 * d * hq
    cu = cu.to(dev)
    maxlen = int((cu[1:] - cu[:-1]).max())
    qkv = torch.randn(T, (hq + 2 * hkv) * d, device=dev).bfloat16()
    q = qkv[:, : hq * d].view(T, hq, d)
    k = qkv[:, hq * d:(hq + hkv) * d].view(T, hkv, d)
    v = qkv[:, (hq + hkv) * d:].view(T, hkv, d)
    do = torch.randn(T, hq, d, device=dev).bfloat16()
    ops = torch.ops.dtg
    scale = 1 / math.sqrt(d)
    o, lse = ops.flash_attn_fwd(q, k, v, cu, maxlen, scale, causal)

    def timeit(fn):
        for _ in range(max(10, a.iters // 2)):  # settle clocks (DVFS) before timing
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.iters):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / a.iters

    tf = timeit(lambda: ops.flash_attn_fwd(q, k, v, cu, maxlen, scale, causal))
    tb = timeit(lambda: ops.flash_attn_bwd_qkv(do, qkv, hq, hkv, d, o, lse, cu, maxlen, scale, causal))
    rec = {"shape": name, "causal": causal, "fwd_ms": tf * 1e3, "bwd_ms": tb * 1e3, "fwd_TFLOPs": causal_flops / tf / 1e12,
           "bwd_TFLOPs": 2.5 * causal_flops / tb / 1e12, "bwd_variant": os.environ.get("DTG_FA_BWD", "split"), "occ": os.environ.get("DTG_FA_OCC", "1")}
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
