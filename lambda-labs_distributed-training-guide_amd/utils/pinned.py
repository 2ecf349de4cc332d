"""Exact-size page-locked host buffers for CPU offload (chapter 05).

`torch.zeros(..., pin_memory=True)` goes through PyTorch's caching host allocator, which rounds
every block up to the next power of two.  For the 405B offload shards that is ruinous: one
rank of an 8-GPU job holds a 101 GB bf16 parameter shard and a 101 GB gradient shard, and each
would be rounded up to 137 GB -- 72 GB of host RAM per rank lost to padding, on a host whose
eight ranks already need ~406 GB each for the offloaded training state.

`pinned_zeros` instead allocates ordinary (pageable) host memory of the exact size and
page-locks it in place with hipHostRegister, so the copy engines DMA straight from / into it
(`non_blocking=True` copies stay asynchronous).  The registration is dropped when the memory
itself is freed (after the device drains), however many views of it are still around until
then.  Without a GPU the buffer is returned pageable; if registration fails, from the caching
allocator.
"""
from __future__ import annotations

import weakref

import torch


def _unregister(ptr: int) -> None:
    # Runs when the buffer's STORAGE is freed (the finalizer hangs on the numpy array the storage
    # keeps alive, not on one tensor object whose views may outlive it).  Drain the device first:
    # an asynchronous copy still reading / writing the pages must not see them unpinned.
    import sys

    if sys.is_finalizing():  # the HIP runtime may already be shutting down: the OS reclaims the pages
        return
    try:
        if torch.cuda.is_initialized():
            torch.cuda.synchronize()
        torch.cuda.cudart().cudaHostUnregister(ptr)
    except Exception:
        pass


def pinned_zeros(n: int, dtype: torch.dtype) -> torch.Tensor:
    n = int(n)
    if n == 0 or not torch.cuda.is_available():
        return torch.zeros(n, dtype=dtype)
    import numpy as np

    esz = torch.empty((), dtype=dtype).element_size()
    arr = np.zeros(n * esz, dtype=np.uint8)  # exact size, zero-filled, pageable
    t = torch.from_numpy(arr).view(dtype)  # shares arr's memory; the storage keeps arr alive
    try:
        rt = torch.cuda.cudart()
        err = rt.cudaHostRegister(t.data_ptr(), n * esz, 0)
        if int(err) != 0:
            raise RuntimeError(f"hipHostRegister returned {int(err)}")
    except Exception:
        return torch.zeros(n, dtype=dtype, pin_memory=True)  # the caching allocator's path
    fin = weakref.finalize(arr, _unregister, t.data_ptr())
    fin.atexit = False  # never at interpreter exit (a synchronize then can hang); process exit frees it
    return t
