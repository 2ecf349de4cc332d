"""Activation checkpointing per decoder layer.

Each layer's forward is re-run inside its backward (non-reentrant torch.utils.checkpoint), so
only the layer inputs stay resident.  The layer's forward is replaced on the instance rather
than wrapped in another module: state-dict names stay unchanged and engine hooks (FSDP
gather/reshard) still fire on the layer's __call__, while the recompute calls the original
forward directly (no hooks, parameters already gathered by the pre-backward node).
"""
import torch
from torch.utils.checkpoint import checkpoint


def apply_activation_checkpointing(model, layers=None, every: int = 1):
    layers = list(layers if layers is not None else model.layers)
    for i, layer in enumerate(layers):
        if i % every:
            continue
        orig = layer.forward

        def fwd(*args, _orig=orig, **kwargs):
            if torch.is_grad_enabled():
                return checkpoint(_orig, *args, use_reentrant=False, **kwargs)
            return _orig(*args, **kwargs)

        layer.forward = fwd
        layer._dtg_checkpointed = True
    return model
