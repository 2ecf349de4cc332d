"""Weight-gradient routing shared by all `dtg` autograd functions.

A parameter managed by a parallel engine carries `main_grad` (a view into the engine's flat
gradient buffer) and `_dtg_notify` (the engine's "this gradient is final for this backward"
callback, used to launch bucketed all-reduce / reduce-scatter while backward continues).
Functions compute a weight gradient straight into `main_grad` -- the first contribution of a
step writes (`out=`), later ones (tied embeddings, gradient accumulation) add -- and return
None to autograd.  Parameters without `main_grad` get an ordinary gradient.
"""
import torch

# When an engine owns the loss (it back-propagates the loss with an implicit gradient of 1 and
# folds any scaling into the optimizer's grad_scale), the fused loss head writes the lm_head
# weight gradient straight into main_grad during its forward pass and skips the grad_output
# multiply in backward: no temporary [V, H] buffer and no extra passes over it.
_DIRECT_LOSS_GRAD = False


def set_direct_loss_grad(enabled: bool):
    global _DIRECT_LOSS_GRAD
    _DIRECT_LOSS_GRAD = bool(enabled)


def direct_loss_grad() -> bool:
    return _DIRECT_LOSS_GRAD


def _fresh(param) -> bool:
    return not getattr(param, "_dtg_grad_written", False)


# While a chunked region back-propagates (parallel/async_tp.py), one weight receives one
# gradient contribution per chunk; the engine must hear "final" once, after the last.
_DEFERRED = None


class deferred_notifications:
    """Collect engine notifications inside the block; fire each parameter's once at exit."""

    def __enter__(self):
        global _DEFERRED
        self.outer, _DEFERRED = _DEFERRED, {}
        return self

    def __exit__(self, *exc):
        global _DEFERRED
        pending, _DEFERRED = _DEFERRED, self.outer
        if exc[0] is None:
            for p in pending.values():
                _mark(p)
        return False


def _mark(param):
    param._dtg_grad_written = True
    if _DEFERRED is not None:
        _DEFERRED[id(param)] = param
        return
    cb = getattr(param, "_dtg_notify", None)
    if cb is not None:
        cb(param)


def route_param_grad(param, grad):
    """Add `grad` into param.main_grad if present; otherwise return it for autograd."""
    mg = getattr(param, "main_grad", None)
    if mg is None:
        return grad
    if _fresh(param):
        mg.copy_(grad.view_as(mg))
    else:
        mg.add_(grad.view_as(mg))
    _mark(param)
    return None


def accumulate_mm_into_main_grad(param, a, b, a_t=None, b_t=None) -> bool:
    """main_grad (+)= a^T @ b without notifying (used by the fused loss head's forward).
    `a_t` / `b_t`: optional contiguous transposes (see route_weight_grad_mm)."""
    mg = getattr(param, "main_grad", None)
    if mg is None:
        return False
    lhs, rhs = (a_t, b_t.t()) if (a_t is not None and b_t is not None) else (a.t(), b)
    if _fresh(param):
        torch.mm(lhs, rhs, out=mg)
        param._dtg_grad_written = True
    else:
        mg.addmm_(lhs, rhs)
    return True


def notify_param(param):
    _mark(param)


def route_weight_grad_mm(param, a, b, a_t=None, b_t=None):
    """Weight gradient a^T @ b (a: [T, out], b: [T, in]) into main_grad without a temporary.

    `a_t` / `b_t` are optional contiguous transposes of a / b ([out, T], [in, T]): given both,
    the GEMM is issued as a_t @ b_t^T, whose operands are both contiguous along the reduction
    (token) dimension -- the layout hipBLASLt runs fastest."""
    if a_t is not None and b_t is not None:
        lhs, rhs = a_t, b_t.t()
    else:
        lhs, rhs = a.t(), b
    mg = getattr(param, "main_grad", None)
    if mg is None:
        return lhs @ rhs
    if _fresh(param):
        torch.mm(lhs, rhs, out=mg)
    else:
        mg.addmm_(lhs, rhs)
    _mark(param)
    return None


def route_embedding_grad(param, ids, dy, num_weights):
    """Embedding backward through the deterministic sorted segment-sum (dtg::embedding_bwd_):
    bitwise reproducible, f32 sums rounded once per row (ATen's index_add_ uses bf16 atomics)."""
    mg = getattr(param, "main_grad", None)
    dy2 = dy.reshape(-1, dy.shape[-1])
    if mg is None:
        g = torch.zeros(num_weights, dy.shape[-1], dtype=dy.dtype, device=dy.device)
        torch.ops.dtg.embedding_bwd_(g, ids.reshape(-1), dy2)
        return g
    if _fresh(param):
        mg.zero_()
    torch.ops.dtg.embedding_bwd_(mg, ids.reshape(-1), dy2)
    _mark(param)
    return None


def reset_grad_state(params):
    for p in params:
        p._dtg_grad_written = False
