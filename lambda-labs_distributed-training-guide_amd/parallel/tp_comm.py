"""Autograd-aware tensor/sequence-parallel collectives.

Activations are token-major [T, H] with T = B*S flattened, so Megatron sequence parallelism
shards dim 0 in contiguous chunks: the sequence all-gather / reduce-scatter pairs map 1:1 onto
RCCL `all_gather_into_tensor` / `reduce_scatter_tensor` with no transposes (the reference's
DTensor `Shard(1)` layouts need a permute around every redistribute).

  gather_seq      fwd all-gather [T/tp,H]->[T,H]      bwd reduce-scatter (sum)
  scatter_seq     fwd reduce-scatter [T,H]->[T/tp,H]  bwd all-gather
  copy_to_tp      fwd identity                        bwd all-reduce (sum)
  reduce_from_tp  fwd all-reduce (sum)                bwd identity
"""
import torch
import torch.distributed as dist

from ..utils import comm


class _GatherSeq(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return comm.all_gather_dim0(x.contiguous(), group)

    @staticmethod
    def backward(ctx, dy):
        return comm.reduce_scatter_dim0(dy.contiguous(), ctx.group), None


class _ScatterSeq(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return comm.reduce_scatter_dim0(x.contiguous(), group)

    @staticmethod
    def backward(ctx, dy):
        return comm.all_gather_dim0(dy.contiguous(), ctx.group), None


class _CopyToTP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return x

    @staticmethod
    def backward(ctx, dy):
        return comm.all_reduce_(dy.contiguous().clone(), ctx.group), None


class _ReduceFromTP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, group):
        return comm.all_reduce_(x.contiguous().clone(), group)

    @staticmethod
    def backward(ctx, dy):
        return dy, None


def gather_seq(x, group):
    return _GatherSeq.apply(x, group)


def scatter_seq(x, group):
    return _ScatterSeq.apply(x, group)


def copy_to_tp(x, group):
    return _CopyToTP.apply(x, group)


def reduce_from_tp(x, group):
    return _ReduceFromTP.apply(x, group)
