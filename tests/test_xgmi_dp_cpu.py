"""Host-side slot bookkeeping of the FSDP gradient pool over xGMI (parallel/xgmi_dp.py) on CPU:
a slot held by a unit whose reduce-scatter has not been issued (the root unit, from its forward
to the end of the backward) is never handed to another unit when the ring wraps, and the choice
depends only on call order (every rank picks the same slot for the same unit)."""
import pytest
import torch

from dtg.parallel.xgmi_dp import XgmiFsdp


def _pool(nslots, slot_numel=8):
    x = object.__new__(XgmiFsdp)
    x.nslots = nslots
    x.device = torch.device("cpu")
    x.slot_numel = slot_numel
    x._pool = torch.zeros(nslots * slot_numel)
    x._free = [None] * nslots
    x._held = [False] * nslots
    x._next = 0
    return x


def _release(x, k):  # the bookkeeping half of reduce_scatter (no GPU work)
    x._held[k] = False


def test_root_slot_is_skipped_when_the_ring_wraps():
    x = _pool(5)
    _, root = x.grad_buffer(8)  # forward: the root unit takes a slot for the whole backward
    order = []
    for _ in range(12):  # 12 decoder units, each reduce-scattered before the next one starts
        _, k = x.grad_buffer(8)
        assert k != root
        order.append(k)
        _release(x, k)
    assert order[:4] == [1, 2, 3, 4] and order[4] == 1  # wraps past the held root slot
    _release(x, root)
    y = _pool(5)  # another rank, same call sequence -> same slots
    _, r2 = y.grad_buffer(8)
    order2 = []
    for _ in range(12):
        _, k = y.grad_buffer(8)
        order2.append(k)
        _release(y, k)
    assert r2 == root and order2 == order


def test_two_units_in_flight_never_share_a_slot():
    x = _pool(5)
    held = set()
    _, root = x.grad_buffer(8)
    held.add(root)
    pending = []
    for _ in range(20):
        _, k = x.grad_buffer(8)
        assert k not in held
        held.add(k)
        pending.append(k)
        if len(pending) > 2:  # max_inflight_rs = 2 reduce-scatters outstanding
            k0 = pending.pop(0)
            _release(x, k0)
            held.discard(k0)


def test_all_slots_held_raises():
    x = _pool(3)
    for _ in range(3):
        x.grad_buffer(8)
    with pytest.raises(RuntimeError, match="slots are held"):
        x.grad_buffer(8)
