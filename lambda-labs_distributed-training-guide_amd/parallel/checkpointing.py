"""Activation checkpointing per decoder layer, with a layer budget.

Each checkpointed layer's forward is re-run inside its backward (non-reentrant
torch.utils.checkpoint), so only the layer inputs stay resident.  The layer's forward is replaced
on the instance rather than wrapped in another module: state-dict names stay unchanged and engine
hooks (FSDP gather/reshard) still fire on the layer's __call__, while the recompute calls the
original forward directly (no hooks, parameters already gathered by the pre-backward node).

The reference checkpoints every decoder layer (/root/reference/05-training-llama-405b/
train_llm.py:122-126).  On a 309 GB (288 GiB) MI355X that leaves most of the HBM idle at 405B
width (the tp 4 x dp 2 one-node recipe peaks at ~157 GB projected to 126 layers), so the number of
checkpointed layers is a knob: `--ac-layers N` checkpoints the first N layers of the rank's stack
and keeps the rest's activations, and `--ac-layers auto` plans N from the measured peaks of the
first two steps against the HBM budget (train/trainer.py `_plan_ac_layers`, with
`layer_activation_bytes` as the first estimate and `ac_layers_for_budget`).  Which layers recompute
changes no value: the recompute is bitwise the forward (tests/test_ac_layers_cpu.py).
"""
import torch
from torch.utils.checkpoint import checkpoint


def _wrap(layer):
    """Install the switchable forward once: checkpointed iff `layer._dtg_checkpointed` at call time."""
    if hasattr(layer, "_dtg_orig_forward"):
        return
    orig = layer.forward
    layer._dtg_orig_forward = orig

    def fwd(*args, _orig=orig, _layer=layer, **kwargs):
        if _layer._dtg_checkpointed and torch.is_grad_enabled():
            return checkpoint(_orig, *args, use_reentrant=False, **kwargs)
        return _orig(*args, **kwargs)

    layer.forward = fwd


def apply_activation_checkpointing(model, layers=None, every: int = 1, count=None):
    """Checkpoint every `every`-th layer of `layers` (default model.layers), and of those only the
    ones among the first `count` layers (None: all)."""
    layers = list(layers if layers is not None else model.layers)
    for i, layer in enumerate(layers):
        _wrap(layer)
        layer._dtg_checkpointed = (i % every == 0) and (count is None or i < count)
    return model


def set_checkpointed_layers(model, count: int, layers=None):
    """Checkpoint exactly the first `count` layers of the stack (the rest keep activations).
    Takes effect from the next forward; must agree across ranks that share collectives inside a
    layer (TP / SP), since a recompute re-issues them."""
    return apply_activation_checkpointing(model, layers, 1, max(0, int(count)))


def checkpointed_count(model, layers=None) -> int:
    layers = list(layers if layers is not None else model.layers)
    return sum(1 for layer in layers if getattr(layer, "_dtg_checkpointed", False))


def layer_activation_bytes(cfg, batch: int, seq: int, tp: int = 1, regather: bool = False) -> int:
    """Bytes one Llama decoder layer keeps for its backward WITHOUT checkpointing, per rank (the
    saved tensors of models/llama.py's fused ops): the two add+RMSNorm residual sums on the
    sequence-parallel shard; the fused QKV, the attention output and LSE and the gate|up output on
    the gathered tokens, column-sharded over TP (SwiGLU's product is recomputed); and the two
    column-parallel GEMM inputs -- gathered, or only this rank's rows with `regather`
    (--sp-regather).  With checkpointing a layer keeps only its input (2 H bytes per local token),
    which the caller subtracts.  Measured at the 405B tp 4 rank, b4 x 4096: 2.23 GB kept /
    1.45 GB re-gathered against 2.50 / 1.70 here (profiles/r6/405b_ac/)."""
    H, I = cfg.hidden_size, cfg.intermediate_size
    nq, nkv, d = cfg.num_attention_heads, cfg.num_key_value_heads, cfg.head_dim
    tp = max(1, int(tp))
    t_full = batch * seq
    t_local = t_full // tp
    norms = 2 * 2 * H * t_local
    cols = 2 * t_full * ((nq + 2 * nkv) * d + nq * d + 2 * I) // tp
    lse = 4 * t_full * nq // tp
    inputs = 2 * 2 * H * (t_local if (regather and tp > 1) else t_full)
    return int(norms + cols + lse + inputs)


def ac_layers_for_budget(n_layers: int, n_ckpt: int, peak_bytes: int, budget_bytes: int, per_layer_bytes: int,
                         input_bytes: int, safety: float = 1.25) -> int:
    """How many of the `n_ckpt` checkpointed layers must STAY checkpointed so that the peak measured
    with them checkpointed (`peak_bytes`) plus the activations the others would keep stays within
    `budget_bytes`.  Each un-checkpointed layer adds per_layer_bytes - input_bytes (times `safety`)."""
    extra = max(1, int((per_layer_bytes - input_bytes) * safety))
    free = budget_bytes - peak_bytes
    release = 0 if free <= 0 else min(n_ckpt, free // extra)
    return int(n_ckpt - release)
