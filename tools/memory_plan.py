#!/usr/bin/env python3
"""Per-GPU memory plan for a model / parallel layout on MI355X (288 GB HBM3E), SURVEY §7.4-§7.5.

Estimates pure-bf16 training state (params, grads, AdamW moments: 8 B/param as in the
reference), the largest gathered FSDP unit, and activations of this framework's Llama layer
(per token per layer: saved norm inputs/outputs, fused QKV, attention output + LSE, gate|up,
SwiGLU output), with or without activation checkpointing and CPU offload.

    python tools/memory_plan.py --model meta-llama/Llama-3.1-405B --world 16 --strategy fsdp --ac
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import dtg  # noqa: E402,F401
from dtg.models import resolve_config  # noqa: E402

HBM_GB = 288.0


def plan(model, world=8, tp=1, strategy="fsdp", batch=1, seq=4096, ac=False, offload=False, resident_params=False,
         ac_layers=None, regather=False):
    """offload: gradients + AdamW state (+ parameters unless resident_params) in host memory;
    resident_params keeps the bf16 parameter shard in HBM and a master copy on the host.
    ac_layers: with `ac`, only that many layers recompute (--ac-layers N); the others keep their
    activations (dtg.parallel.checkpointing.layer_activation_bytes, with --sp-regather)."""
    c = resolve_config(model)
    P = c.num_params()
    H, I, L = c.hidden_size, c.intermediate_size, c.num_hidden_layers
    nq, nkv, d = c.num_attention_heads, c.num_key_value_heads, c.head_dim
    dp = world // tp
    p_local = P / tp
    gb = 1e9
    if strategy == "ddp":
        params, grads, opt = 2 * p_local, 2 * p_local, 4 * p_local
    elif strategy == "zero":
        params, grads, opt = 2 * p_local, 2 * p_local, 4 * p_local / dp
    else:  # fsdp
        params, grads, opt = 2 * p_local / dp, 2 * p_local / dp, 4 * p_local / dp
    unit = 2 * (H * (nq + 2 * nkv) * d + nq * d * H + 3 * H * I + 2 * H) / tp
    gather = 2 * unit if strategy == "fsdp" else 0  # current + prefetched unit (grads: one more in bwd)
    T = batch * seq / (tp if tp > 1 else 1)  # sequence-parallel shard of the norm/residual stream
    Tfull = batch * seq
    per_tok_layer = 2 * (4 * H / (tp if tp > 1 else 1)) + 2 * Tfull / T * ((nq + 2 * nkv) * d + nq * d + 3 * I) / tp
    acts = L * T * per_tok_layer if not ac else L * T * 2 * H + T * per_tok_layer
    if ac and ac_layers is not None:  # the planner the trainer uses: kept layers' saved tensors
        from dtg.parallel.checkpointing import layer_activation_bytes

        n_ckpt = max(0, min(L, int(ac_layers)))
        kept = layer_activation_bytes(c, batch, seq, tp, regather)
        acts = n_ckpt * T * 2 * H + (L - n_ckpt) * kept + T * per_tok_layer
    logits = 2 * min(Tfull, (1 << 29) // max(c.vocab_size, 1)) * c.vocab_size / tp * 2
    host = 0.0
    if offload:
        host = params + grads + opt
        grads = opt = 0.0
        if not resident_params:
            params = 0.0
    total = params + grads + opt + gather + acts + logits
    return {
        "model": c.hf_name or model, "params_B": P / 1e9, "world": world, "tp": tp, "dp": dp, "strategy": strategy,
        "params_gb": params / gb, "grads_gb": grads / gb, "adamw_gb": opt / gb, "gathered_units_gb": gather / gb,
        "activations_gb": acts / gb, "loss_chunk_gb": logits / gb, "total_gb_per_gpu": total / gb,
        "host_gb_per_gpu": host / gb, "fits_288gb": total / gb < HBM_GB * 0.92,
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="meta-llama/Llama-3.1-405B")
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--tp", type=int, default=1)
    ap.add_argument("--strategy", choices=["ddp", "zero", "fsdp"], default="fsdp")
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--seq", type=int, default=4096)
    ap.add_argument("--ac", action="store_true")
    ap.add_argument("--offload", action="store_true")
    ap.add_argument("--resident-params", action="store_true",
                    help="with --offload: parameter shard stays in HBM (--offload-params off / auto)")
    ap.add_argument("--ac-layers", type=int, default=None, help="with --ac: layers that recompute (the rest keep)")
    ap.add_argument("--regather", action="store_true", help="--sp-regather: kept layers hold local GEMM inputs")
    ap.add_argument("--exact", action="store_true",
                    help="also print the exact FSDP unit layout (dtg.parallel.plan on a meta-device model)")
    a = ap.parse_args()
    r = plan(a.model, a.world, a.tp, a.strategy, a.batch, a.seq, a.ac, a.offload, a.resident_params, a.ac_layers,
             a.regather)
    for k, v in r.items():
        print(f"{k:20s} {v:.2f}" if isinstance(v, float) else f"{k:20s} {v}")
    if a.exact and a.tp == 1:
        from dtg.models import build_model
        from dtg.parallel.plan import fsdp_plan

        fp = fsdp_plan(build_model(a.model, device="meta", init=False), a.world)
        print(f"{'fsdp_units':20s} {len(fp.units)} + root")
        print(f"{'shard_elems/rank':20s} {fp.shard_numel}")
        print(f"{'state_gb/rank':20s} {fp.per_rank_state_bytes() / 1e9:.2f}")
        print(f"{'largest_gather_gb':20s} {fp.largest_gather_bytes() / 1e9:.3f}")
        print(f"{'padding':20s} {100 * fp.padding_fraction():.4f} %")


if __name__ == "__main__":
    main()
