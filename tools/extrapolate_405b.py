#!/usr/bin/env python3
"""Llama-3.1-405B step time per GPU from the chapter-05 engine at exact width, reduced depth.

Inputs: chapter-05 logs (`05-training-llama-405b/train_llm.py`, b1 x 4096, transformer wrap +
activation checkpointing) at depths 2 and 4 on one MI355X, with CPU offload (gradients + AdamW
state on the host, native host AdamW under the backward) and without it.  Per-layer costs are
the depth-4 minus depth-2 difference / 2; the rest is the fixed cost (embedding, loss head).

From those it projects the per-GPU step of the full 126-layer model on 64 GPUs (the reference's
8 x 8 cluster, BASELINE row 9: 30 s/step = 136.5 tok/s/GPU) for two recipes.  Everything that
is not measured here is an ASSUMPTION printed with the result (this box has one GPU):

  A  the reference's recipe: FULL_SHARD over all 64 GPUs + CPU offload.  Every layer's
     parameters are all-gathered twice (forward, backward recompute) and its gradients
     reduce-scattered once across the 64 GPUs, i.e. over the inter-node network.
  B  the MI355X-native recipe: HYBRID_SHARD inside each node (8-way, xGMI) with the optimizer
     state offloaded (params + grads resident: 4 B/param / 8 = 203 GB of 288 GB), replicas
     across the 8 nodes; per layer the gathers / scatters run over xGMI, and the inter-node
     traffic is one all-reduce of each GPU's gradient shard per step, issued per unit inside
     the backward (parallel/fsdp.py).

    python tools/extrapolate_405b.py gpurun_out/r3_s03 [--net-gbs 50 --xgmi-gbs 300]
"""
import argparse
import ast
import json
import os
import re
import statistics

FULL_DEPTH = 126
PARAMS_LAYER = 16384 * (16384 + 2 * 1024) + 16384 * 16384 + 3 * 16384 * 53248 + 2 * 16384  # 3.187e9
PARAMS_TOTAL = 405.85e9
TOKENS = 4096
REF_TOK_S_GPU = 136.5


def phases(path):
    recs = []
    for line in open(path):
        m = re.search(r"(\{'global_step'.*\})", line)
        if m:
            try:
                recs.append(ast.literal_eval(m.group(1)))
            except (ValueError, SyntaxError):
                pass
    recs = [r for r in recs if r.get("global_step", 0) >= 3] or recs  # skip warmup steps
    out = {}
    for k in ("time/forward", "time/backward", "time/update", "time/total"):
        vals = [r[k] for r in recs if k in r]
        out[k] = statistics.median(vals) if vals else float("nan")
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--net-gbs", type=float, default=50.0, help="ASSUMED inter-node bandwidth per GPU (GB/s)")
    ap.add_argument("--xgmi-gbs", type=float, default=300.0, help="ASSUMED RCCL intra-node bus bandwidth (GB/s)")
    ap.add_argument("--host-gbs", type=float, default=347.0, help="host AdamW GB/s (profiles/r2/s15_host_adamw.log)")
    ap.add_argument("--world", type=int, default=64)
    ap.add_argument("--per-node", type=int, default=8)
    a = ap.parse_args()
    d = a.dir
    no2, no4 = phases(os.path.join(d, "ch05_405b_d2_no_offload.log")), phases(os.path.join(d, "ch05_405b_d4_no_offload.log"))
    of2, of4 = phases(os.path.join(d, "ch05_405b_d2.log")), phases(os.path.join(d, "ch05_405b_d4.log"))
    lay = {k: (no4[k] - no2[k]) / 2 for k in no2}
    fixed = {k: no2[k] - 2 * lay[k] for k in no2}
    lay_off = {k: (of4[k] - of2[k]) / 2 for k in of2}
    comp_layer = lay["time/forward"] + lay["time/backward"]  # ms, GPU compute incl. AC recompute
    comp_fixed = fixed["time/forward"] + fixed["time/backward"]
    compute_s = (FULL_DEPTH * comp_layer + comp_fixed) / 1e3
    bytes_layer = 2 * PARAMS_LAYER
    # offload cost per layer at W=1: the backward's extra time over the no-offload run
    off_extra_ms = lay_off["time/backward"] + lay_off["time/update"] - lay["time/backward"] - lay["time/update"]
    W, G = a.world, a.per_node
    # A: FULL_SHARD over W, network-bound gathers / scatters, offload of 1/W
    comm_a_layer = 3 * bytes_layer * (W - 1) / W / (a.net_gbs * 1e9) * 1e3
    layer_a = max(comp_layer, comm_a_layer)
    host_a = PARAMS_TOTAL / W * 14 / (a.host_gbs * 1e9)
    step_a = (FULL_DEPTH * layer_a + comp_fixed) / 1e3 + host_a * 0.0  # host update overlaps the backward
    # B: HYBRID in node (G-way shard, xGMI), replicas across nodes, optimizer state offloaded
    comm_b_layer = 3 * bytes_layer * (G - 1) / G / (a.xgmi_gbs * 1e9) * 1e3
    layer_b = max(comp_layer, comm_b_layer)
    R = W // G
    ar_s = 2 * (R - 1) / R * (2 * PARAMS_TOTAL / G) / (a.net_gbs * 1e9)
    bwd_s = FULL_DEPTH * (lay["time/backward"]) / 1e3
    host_b = PARAMS_TOTAL / G * 14 / (a.host_gbs * 1e9)
    exposed_b = max(0.0, ar_s - bwd_s) + max(0.0, host_b - bwd_s)
    step_b = (FULL_DEPTH * layer_b + comp_fixed) / 1e3 + exposed_b
    res = {
        "metric": "Llama-3.1-405B step per GPU, projected from exact-width chapter-05 layers (1 MI355X)",
        "measured": {"layer_fwd_ms": round(lay["time/forward"], 1), "layer_bwd_ms": round(lay["time/backward"], 1),
                     "layer_compute_ms": round(comp_layer, 1), "fixed_compute_ms": round(comp_fixed, 1),
                     "layer_offload_extra_ms_at_W1": round(off_extra_ms, 1),
                     "compute_only_step_s": round(compute_s, 2),
                     "compute_only_tok_s_gpu": round(TOKENS / compute_s, 1)},
        "assumptions": {"net_GBps_per_gpu": a.net_gbs, "xgmi_bus_GBps": a.xgmi_gbs, "host_adamw_GBps": a.host_gbs,
                        "world": W, "gpus_per_node": G},
        "A_full_shard_offload": {"comm_per_layer_ms": round(comm_a_layer, 1), "step_s": round(step_a, 2),
                                 "tok_s_gpu": round(TOKENS / step_a, 1), "vs_reference": round(TOKENS / step_a / REF_TOK_S_GPU, 3)},
        "B_hybrid_xgmi_optimizer_offload": {"comm_per_layer_ms": round(comm_b_layer, 1),
                                            "inter_node_allreduce_s": round(ar_s, 2), "host_adamw_s": round(host_b, 2),
                                            "exposed_s": round(exposed_b, 2), "step_s": round(step_b, 2),
                                            "tok_s_gpu": round(TOKENS / step_b, 1),
                                            "vs_reference": round(TOKENS / step_b / REF_TOK_S_GPU, 3)},
        "reference_tok_s_gpu": REF_TOK_S_GPU,
    }
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
