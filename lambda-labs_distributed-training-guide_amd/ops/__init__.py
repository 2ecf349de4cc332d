"""Hot-path operators: autograd-aware wrappers over the `dtg` library.

GPU tensors run the gfx950 HIP kernels from `_C.so`; CPU tensors run the f32 references in
`_cpu.py` (PyTorch device dispatch, no per-op backend switch).  GEMMs are hipBLASLt via
`torch.mm`.  Weight gradients are routed through `grad_routing`, so the parallel engines can
receive them directly in flat communication buffers (`param.main_grad`) with a per-parameter
ready notification, instead of through `.grad` accumulation.
"""
from . import _schema  # noqa: F401  (defines the operator schemas)
from . import _cpu  # noqa: F401  (CPU implementations)
from . import _native

_native.load()
if not _native.LOADED:  # CPU-only box without a build: host AdamW falls back to the f32 reference
    _schema.LIB.impl("adamw_cpu_", lambda p, g, m, v, lr, b1, b2, eps, wd, step, gs: _cpu.adamw_(
        p, None, g, m, v, lr, b1, b2, eps, wd, step, gs), "CPU")

from .functional import (  # noqa: E402
    add_rms_norm,
    attention,
    embedding,
    fused_linear_cross_entropy,
    linear,
    rms_norm,
    rope,
    rope_tables,
    swiglu,
    swiglu_mlp,
    vocab_parallel_fused_linear_cross_entropy,
)
from .grad_routing import route_param_grad  # noqa: E402
from .adamw import adamw_step  # noqa: E402

import contextlib as _contextlib  # noqa: E402

import torch as _torch  # noqa: E402


@_contextlib.contextmanager
def fa_tuning(device="cuda", kv_split: int = -1, kv_qb: int = -1):
    """Set the flash-attention backward's launch tuning (dK/dV query-item split, 0 = auto; dK/dV
    query rows per item, 32 | 64) for the duration of the block.  The kernels read these from
    DTG_FA_KV_SPLIT / DTG_FA_KV_QB once, when the extension loads, never per launch."""
    like = _torch.empty(0, device=device)
    old = _torch.ops.dtg.flash_attn_tuning(like, kv_split, kv_qb)
    try:
        yield
    finally:
        _torch.ops.dtg.flash_attn_tuning(like, old[0], old[1])

__all__ = [
    "add_rms_norm", "attention", "rope", "embedding", "fused_linear_cross_entropy", "linear", "rms_norm",
    "rope_tables", "swiglu", "swiglu_mlp", "vocab_parallel_fused_linear_cross_entropy", "route_param_grad", "adamw_step",
    "fa_tuning",
]
