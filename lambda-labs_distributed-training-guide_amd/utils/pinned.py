"""Exact-size page-locked host buffers for CPU offload (chapter 05).

`torch.zeros(..., pin_memory=True)` goes through PyTorch's caching host allocator, which rounds
every block up to the next power of two.  For the 405B offload shards that is ruinous: one
rank of an 8-GPU job holds a 101 GB bf16 parameter shard and a 101 GB gradient shard, and each
would be rounded up to 137 GB -- 72 GB of host RAM per rank lost to padding, on a host whose
eight ranks already need ~406 GB each for the offloaded training state.

`pinned_zeros` instead allocates ordinary (pageable) host memory of the exact size and
page-locks it in place with hipHostRegister, so the copy engines DMA straight from / into it
(`non_blocking=True` copies stay asynchronous).  The registration is dropped when the tensor
object is collected.  Without a GPU (or if registration fails) the buffer is returned pageable.
"""
from __future__ import annotations

import weakref

import torch


def _unregister(ptr: int) -> None:
    try:
        torch.cuda.cudart().cudaHostUnregister(ptr)
    except Exception:
        pass


def pinned_zeros(n: int, dtype: torch.dtype) -> torch.Tensor:
    t = torch.zeros(int(n), dtype=dtype)
    if n == 0 or not torch.cuda.is_available():
        return t
    try:
        rt = torch.cuda.cudart()
        err = rt.cudaHostRegister(t.data_ptr(), t.numel() * t.element_size(), 0)
        if int(err) != 0:
            raise RuntimeError(f"hipHostRegister returned {int(err)}")
    except Exception:
        return torch.zeros(int(n), dtype=dtype, pin_memory=True)  # the caching allocator's path
    weakref.finalize(t, _unregister, t.data_ptr())
    return t
