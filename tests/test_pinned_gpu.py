"""Exact-size page-locked host buffers for the offload shards (dtg.utils.pinned)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_pinned_zeros_exact_size_and_async_copies(cuda):
    from dtg.utils.pinned import pinned_zeros

    n = 3 * (1 << 20) + 7  # not a power of two
    h = pinned_zeros(n, torch.bfloat16)
    assert h.is_pinned() and h.numel() == n and h.untyped_storage().nbytes() == 2 * n
    assert torch.count_nonzero(h) == 0
    d = torch.randn(n, device=cuda).bfloat16()
    h.copy_(d, non_blocking=True)
    torch.cuda.synchronize()
    back = torch.empty_like(d)
    back.copy_(h, non_blocking=True)
    torch.cuda.synchronize()
    assert torch.equal(back, d)


def test_pinned_view_outlives_the_tensor_object(cuda):
    """The registration belongs to the memory, not to the first tensor object: a view kept after
    the original tensor is gone is still page-locked (async copies stay DMA), and the pages are
    unpinned only when the last view is freed."""
    import gc

    from dtg.utils.pinned import pinned_zeros

    h = pinned_zeros(1 << 20, torch.bfloat16)
    v = h[4096:8192]
    del h
    gc.collect()
    assert v.is_pinned()
    d = torch.randn(4096, device=cuda).bfloat16()
    v.copy_(d, non_blocking=True)
    torch.cuda.synchronize()
    assert torch.equal(v.to(cuda), d)
