"""Learning-rate scaling with the effective batch size.

effective batch = per-GPU batch x data-parallel size x gradient-accumulation steps; when it
changes by a factor k, scale the LR linearly (SGD-style) or by sqrt(k) (Adam-style)."""
import math


def effective_batch(batch_size: int, dp_size: int, grad_accum: int = 1) -> int:
    return batch_size * dp_size * grad_accum


def scale_lr(base_lr: float, base_batch: int, new_batch: int, rule: str = "sqrt") -> float:
    k = new_batch / base_batch
    if rule == "linear":
        return base_lr * k
    if rule == "sqrt":
        return base_lr * math.sqrt(k)
    raise ValueError(rule)
