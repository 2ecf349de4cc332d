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

__all__ = [
    "add_rms_norm", "attention", "rope", "embedding", "fused_linear_cross_entropy", "linear", "rms_norm",
    "rope_tables", "swiglu", "swiglu_mlp", "vocab_parallel_fused_linear_cross_entropy", "route_param_grad", "adamw_step",
]
