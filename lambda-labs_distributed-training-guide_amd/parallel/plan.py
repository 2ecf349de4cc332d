"""Sharding plans without hardware: the exact FSDP unit layout that
`FullyShard` builds -- units, padded flat sizes, per-rank shard sizes -- computed from a model
on the meta device, so 405B layouts at W = 64..512 can be inspected (and tested against the
engine under a fake process group) on a laptop.
"""
from __future__ import annotations

import dataclasses
from typing import List

import torch.nn as nn

from .fsdp import ALIGN, _round_up, size_based_units, transformer_units


@dataclasses.dataclass
class UnitPlan:
    name: str
    numel: int          # real parameter elements
    padded_numel: int   # flat buffer length (each param 16-aligned, total a multiple of world*16)
    shard_numel: int    # per-rank slice

    def gather_bytes(self, elem_bytes: int = 2) -> int:
        return self.padded_numel * elem_bytes


@dataclasses.dataclass
class FsdpPlan:
    world: int
    units: List[UnitPlan]
    root: UnitPlan

    @property
    def all_units(self):
        return self.units + [self.root]

    @property
    def shard_numel(self) -> int:
        return sum(u.shard_numel for u in self.all_units)

    @property
    def total_params(self) -> int:
        return sum(u.numel for u in self.all_units)

    def per_rank_state_bytes(self, param_bytes=2, grad_bytes=2, state_bytes=2) -> int:
        """params + grads + 2 AdamW moments of this rank's shard (pure bf16: 8 B/element)."""
        return self.shard_numel * (param_bytes + grad_bytes + 2 * state_bytes)

    def largest_gather_bytes(self, elem_bytes: int = 2) -> int:
        return max(u.gather_bytes(elem_bytes) for u in self.units) if self.units else 0

    def padding_fraction(self) -> float:
        return self.shard_numel * self.world / max(1, self.total_params) - 1.0


def _unit_plan(name, params, world) -> UnitPlan:
    cur = 0
    for p in params:
        cur += _round_up(p.numel(), ALIGN)
    padded = _round_up(max(cur, 1), world * ALIGN)
    return UnitPlan(name, sum(p.numel() for p in params), padded, padded // world)


def fsdp_plan(model: nn.Module, world: int, policy: str = "transformer", min_num_params: int = 100_000_000) -> FsdpPlan:
    """Same unit selection and padding as FullyShard.__init__ (parallel/fsdp.py)."""
    mods = transformer_units(model) if policy == "transformer" else size_based_units(model, min_num_params)
    names = {id(m): n for n, m in model.named_modules()}
    seen = set()
    units = []
    for m in mods:
        ps = [p for _, p in m.named_parameters() if id(p) not in seen and p.requires_grad]
        for p in ps:
            seen.add(id(p))
        if ps:
            units.append(_unit_plan(names.get(id(m), "?"), ps, world))
    root = [p for _, p in model.named_parameters() if id(p) not in seen and p.requires_grad]
    return FsdpPlan(world, units, _unit_plan("<root>", root, world))
