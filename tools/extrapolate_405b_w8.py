#!/usr/bin/env python3
"""Llama-3.1-405B on ONE 8-GPU MI355X node: per-rank step model from two measured depths.

Input: chapter-05 logs of rank 0 of the W = 8 job (`tools/run_405b_node_w8.sh`: DTG_FAKE_WORLD=8,
exact 405B width, b1 x 4096, FSDP transformer wrap + activation checkpointing, CPU offload with
the parameter shard resident in HBM, 16 CPUs, host AdamW under the backward) at two depths.
Per-layer costs = difference / depth difference; the rest is the fixed cost (embedding, loss
head, root unit).  The 126-layer step, memory and traffic are extrapolated linearly.

What one GPU cannot measure is modelled, with every assumption printed:
  * the FSDP collectives over xGMI (per layer and rank: parameter all-gather in the forward and
    again for the backward recompute, gradient reduce-scatter: 3 x 7/8 x 6.37 GB), at an
    ASSUMED bus bandwidth (--xgmi-gbs; the bench's N > 1 collective sweep measures it), either
    hidden under the layer's compute or fully exposed (the two bounds);
  * the node's DRAM shared by 8 ranks (host AdamW streams 14 B per parameter, plus the gradient
    D2H and parameter H2D), at an ASSUMED node DRAM bandwidth (--dram-gbs).

    python tools/extrapolate_405b_w8.py gpurun_out/r4_s02 [--xgmi-gbs 300 --dram-gbs 900]
"""
import argparse
import ast
import glob
import json
import os
import re
import statistics

FULL_DEPTH = 126
W = 8
PARAMS_LAYER = 16384 * (16384 + 2 * 1024) + 16384 * 16384 + 3 * 16384 * 53248 + 2 * 16384  # 3.187e9
PARAMS_ROOT = 2 * 128256 * 16384 + 16384
TOKENS = 4096
REF_TOK_S_GPU = 136.5


def records(path):
    recs = []
    for line in open(path):
        m = re.search(r"(\{'global_step'.*\})", line)
        if m:
            try:
                recs.append(ast.literal_eval(m.group(1)))
            except (ValueError, SyntaxError):
                pass
    return [r for r in recs if r.get("global_step", 0) >= 3] or recs


def med(recs, k):
    vals = [r[k] for r in recs if k in r]
    return statistics.median(vals) if vals else float("nan")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--xgmi-gbs", type=float, default=300.0, help="ASSUMED RCCL all-gather/reduce-scatter bus GB/s")
    ap.add_argument("--dram-gbs", type=float, default=900.0, help="ASSUMED sustained node DRAM GB/s (8 ranks share it)")
    ap.add_argument("--json", action="store_true")
    a = ap.parse_args()
    runs = {}
    for f in glob.glob(os.path.join(a.dir, "ch05_405b_w8_rank0_depth*.log")):
        d = int(re.search(r"depth(\d+)", f).group(1))
        recs = records(f)
        if recs:
            runs[d] = {k: med(recs, k) for k in ("time/forward", "time/backward", "time/update", "time/total",
                                                  "peak_alloc_in_gb", "offload/host_adamw_s", "offload/host_adamw_gbs",
                                                  "offload/d2h_gb", "offload/d2h_gbs", "offload/h2d_gbs",
                                                  "host/rss_gb", "host/pinned_gb")}
    if len(runs) < 2:
        raise SystemExit(f"need logs at two depths in {a.dir}, found {sorted(runs)}")
    lo, hi = min(runs), max(runs)
    per = {k: (runs[hi][k] - runs[lo][k]) / (hi - lo) for k in runs[hi]}
    full = {k: runs[hi][k] + per[k] * (FULL_DEPTH - hi) for k in runs[hi]}
    fwd, bwd, upd = full["time/forward"] / 1e3, full["time/backward"] / 1e3, full["time/update"] / 1e3
    compute = fwd + bwd + upd
    # FSDP traffic over xGMI per layer and rank (bytes received): AG fwd + AG bwd recompute + RS
    layer_bytes = 3 * (W - 1) / W * PARAMS_LAYER * 2
    comm_layer = layer_bytes / (a.xgmi_gbs * 1e9)
    comm = FULL_DEPTH * comm_layer + 3 * (W - 1) / W * PARAMS_ROOT * 2 / (a.xgmi_gbs * 1e9)
    layer_compute = (per["time/forward"] + per["time/backward"]) / 1e3
    # node DRAM: 8 ranks x (host AdamW 14 B/param + D2H grads 2 B + H2D params 2 B) per step
    params_rank = (FULL_DEPTH * PARAMS_LAYER + PARAMS_ROOT) / W
    dram_bytes_node = W * params_rank * 18
    dram_s = dram_bytes_node / (a.dram_gbs * 1e9)
    hidden = max(compute, dram_s)
    exposed = max(compute + comm, dram_s)
    host_state_rank = params_rank * 8 / 1e9
    host_state_rank_ring = params_rank * 6 / 1e9
    out = {
        "measured_depths": sorted(runs),
        "measured": runs,
        "per_layer": {"forward_ms": per["time/forward"], "backward_ms": per["time/backward"],
                      "hbm_gb": per["peak_alloc_in_gb"], "host_rss_gb": per["host/rss_gb"],
                      "host_adamw_s": per["offload/host_adamw_s"], "d2h_gb": per["offload/d2h_gb"]},
        "full_126": {"forward_s": fwd, "backward_s": bwd, "update_s": upd, "compute_step_s": compute,
                     "peak_hbm_gb": full["peak_alloc_in_gb"], "host_adamw_s": full["offload/host_adamw_s"],
                     "d2h_gb": full["offload/d2h_gb"],
                     "host_state_gb_per_rank": host_state_rank, "host_state_gb_per_rank_grad_ring": host_state_rank_ring,
                     "host_state_tb_per_node": W * host_state_rank / 1e3,
                     "host_state_tb_per_node_grad_ring": W * host_state_rank_ring / 1e3},
        "xgmi_model": {"assumed_busbw_gbs": a.xgmi_gbs, "gb_per_layer_rank": layer_bytes / 1e9,
                       "comm_per_layer_s": comm_layer, "compute_per_layer_s": layer_compute,
                       "comm_step_s": comm},
        "dram_model": {"assumed_node_dram_gbs": a.dram_gbs, "node_bytes_per_step_tb": dram_bytes_node / 1e12,
                       "dram_step_s": dram_s},
        "step_s": {"comm_hidden": hidden, "comm_exposed": exposed},
        "tok_s_per_gpu": {"comm_hidden": TOKENS / hidden, "comm_exposed": TOKENS / exposed,
                          "reference_64xH100": REF_TOK_S_GPU},
    }
    if a.json:
        print(json.dumps(out, indent=1))
        return
    print(f"| depth | fwd s | bwd s | update s | step s | peak HBM GB | host AdamW s (GB/s) | D2H GB (GB/s) | H2D GB/s | host RSS GB | pinned GB |")
    print("|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|")
    for d in sorted(runs):
        r = runs[d]
        print(f"| {d} | {r['time/forward'] / 1e3:.3f} | {r['time/backward'] / 1e3:.3f} | {r['time/update'] / 1e3:.3f} | "
              f"{r['time/total'] / 1e3:.3f} | {r['peak_alloc_in_gb']:.1f} | {r['offload/host_adamw_s']:.2f} "
              f"({r['offload/host_adamw_gbs']:.0f}) | {r['offload/d2h_gb']:.1f} ({r['offload/d2h_gbs']:.1f}) | "
              f"{r['offload/h2d_gbs']:.1f} | {r['host/rss_gb']:.0f} | {r['host/pinned_gb']:.0f} |")
    print(f"| **126 (extrapolated)** | {fwd:.2f} | {bwd:.2f} | {upd:.2f} | {compute:.2f} | {full['peak_alloc_in_gb']:.0f} | "
          f"{full['offload/host_adamw_s']:.2f} | {full['offload/d2h_gb']:.0f} | | | |")
    print()
    print(f"per layer: fwd {per['time/forward']:.1f} ms, bwd {per['time/backward']:.1f} ms, HBM {per['peak_alloc_in_gb']:.2f} GB, "
          f"host RSS {per['host/rss_gb']:.2f} GB")
    print(f"host state per rank at 126 layers: {host_state_rank:.0f} GB (8 B/param), {host_state_rank_ring:.0f} GB with the "
          f"gradient ring (6 B/param); per node x8: {W * host_state_rank / 1e3:.2f} / {W * host_state_rank_ring / 1e3:.2f} TB")
    print(f"xGMI (ASSUMED {a.xgmi_gbs:.0f} GB/s bus): {layer_bytes / 1e9:.1f} GB per layer per rank = {comm_layer * 1e3:.0f} ms vs "
          f"{layer_compute * 1e3:.0f} ms of compute per layer; {comm:.1f} s per step if fully exposed")
    print(f"node DRAM (ASSUMED {a.dram_gbs:.0f} GB/s): {dram_bytes_node / 1e12:.2f} TB per step = {dram_s:.1f} s")
    print(f"step: {hidden:.1f} s (collectives hidden) .. {exposed:.1f} s (exposed) -> "
          f"{TOKENS / hidden:.0f} .. {TOKENS / exposed:.0f} tok/s/GPU vs reference {REF_TOK_S_GPU}")


if __name__ == "__main__":
    main()
