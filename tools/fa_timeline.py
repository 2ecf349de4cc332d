#!/usr/bin/env python3
"""Where a flash-attention forward launch spends its time, from in-kernel stamps.

`flash_attn_fwd_stamped` records per work item (100 MHz s_memrealtime ticks): start, prologue
done (Q + first K/V tile staged), tile loop done, output stores complete (the stamped build
waits for them, so its span is an upper bound: use `plain_ms` for the real time), plus the
hardware wave id / XCC id of the workgroup that ran it.  This prints, per shape: the launch span, the mean prologue / loop / epilogue
per workgroup, the loop time per K/V tile, and CU-slot utilisation (resident workgroups per CU
over the span, vs. the 2 the kernel's occupancy allows), i.e. how much of the span is per-item
overhead, how much is tail and how much is the tile loop itself.

    python tools/fa_timeline.py            # S = 512 / 1024 / 8192, causal and not
"""
import json
import math
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

import dtg  # noqa: E402,F401
import dtg.ops  # noqa: E402,F401

TICK_NS = 10.0


def run(S, causal, hq=32, hkv=8, d=128, tokens=16384):
    dev = torch.device("cuda:0")
    B = tokens // S
    T = B * S
    cu = torch.arange(0, T + 1, S, dtype=torch.int32, device=dev)
    qkv = torch.randn(T, (hq + 2 * hkv) * d, device=dev).bfloat16()
    q = qkv[:, : hq * d].view(T, hq, d)
    k = qkv[:, hq * d:(hq + hkv) * d].view(T, hkv, d)
    v = qkv[:, (hq + hkv) * d:].view(T, hkv, d)
    scale = 1 / math.sqrt(d)
    ops = torch.ops.dtg
    for _ in range(20):
        ops.flash_attn_fwd(q, k, v, cu, S, scale, causal)
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(20):
        ops.flash_attn_fwd(q, k, v, cu, S, scale, causal)
    ev1.record()
    torch.cuda.synchronize()
    plain_ms = ev0.elapsed_time(ev1) / 20
    for _ in range(5):
        _, _, st = ops.flash_attn_fwd_stamped(q, k, v, cu, S, scale, causal)
    torch.cuda.synchronize()
    st = st.cpu()
    ok = st[:, 0] > 0
    st = st[ok]
    t0, t1, t2, t3 = (st[:, i].double() for i in range(4))
    hw, xcc = st[:, 4], st[:, 5]
    span = (t3.max() - t0.min()).item() * TICK_NS / 1e3
    cu_id = (hw >> 8) & 0xF
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 0x7
    slot = ((xcc & 0xF) * 1000 + se * 100 + sh * 16 + cu_id).tolist()
    ncu = len(set(slot))
    busy = (t3 - t0).sum().item() * TICK_NS / 1e3  # workgroup-µs
    util = busy / (span * ncu * 2)
    nqb = (S + 127) // 128
    # tiles per item from its index (z slowest; causal: heavy first)
    items = torch.nonzero(ok).flatten()
    z = items // (hq * B)
    qb = (nqb - 1 - z) if causal else z
    tiles = torch.minimum(torch.full_like(qb, S), (qb + 1) * 128) // 64 if causal else torch.full_like(qb, S // 64)
    loop_us = (t2 - t1) * TICK_NS / 1e3
    rec = {
        "S": S, "causal": causal, "plain_ms": round(plain_ms, 4), "span_us": round(span, 1),
        "items": int(len(st)), "cus_seen": ncu,
        "mean_prologue_us": round(((t1 - t0).mean() * TICK_NS / 1e3).item(), 2),
        "mean_loop_us": round(loop_us.mean().item(), 2),
        "mean_epilogue_us": round(((t3 - t2).mean() * TICK_NS / 1e3).item(), 2),
        "loop_us_per_tile": round((loop_us / tiles.double()).mean().item(), 3),
        "slot_utilisation": round(util, 3),
        "tail_us": round(((t3.max() - t0.max()) * TICK_NS / 1e3).item(), 1),
    }
    print(json.dumps(rec), flush=True)


def main():
    for S in (512, 1024, 8192):
        for causal in (True, False):
            run(S, causal)


if __name__ == "__main__":
    main()
