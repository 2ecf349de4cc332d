"""Functional fused AdamW over flat buffers (HIP kernel on GPU, reference on CPU)."""
import torch


def adamw_step(p, g, m, v, *, lr, step, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.01,
               grad_scale=1.0, master=None, hyper=None):
    """One torch-fused-AdamW-equivalent update of flat buffers (in place).

    p: bf16 params; g: grads (bf16/f32); m, v: states (bf16 as in the reference, or f32);
    master: optional f32 master copy of p; grad_scale multiplies g first (DP averaging,
    gradient-accumulation division, clipping) so no separate scaling pass is needed.
    hyper: optional device f32 [lr, 1 - beta1^step, sqrt(1 - beta2^step)] read by the kernel
    instead of `lr` / `step` (HIP-graph replays, see dtg.train.graph)."""
    torch.ops.dtg.adamw_(p, master, g, m, v, float(lr), float(beta1), float(beta2), float(eps),
                         float(weight_decay), int(step), float(grad_scale), hyper)


def adamw_step_cpu(p, g, m, v, *, lr, step, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.01, grad_scale=1.0):
    """Host AdamW on pinned CPU shards (FSDP CPU offload): native OpenMP C++ kernel."""
    torch.ops.dtg.adamw_cpu_(p, g, m, v, float(lr), float(beta1), float(beta2), float(eps), float(weight_decay),
                             int(step), float(grad_scale))
