"""Ulysses sequence parallelism (contiguous sequence slices, all-to-all seq<->heads around the
ordinary varlen flash attention) == the unsharded model, on gloo ranks: the all-to-all pair
round-trips, attention matches, and Llama training (dense and packed rows, GQA with kv heads
fewer than ranks) produces the single-process parameters."""
import pytest
import torch

import dtg  # noqa: F401
import dtg.ops  # noqa: F401  (registers torch.ops.dtg)

from _dist import run_distributed


def _roundtrip(rank, world):
    from dtg.parallel.ulysses import _head_to_seq, _seq_to_head

    B, s, C = 2, 3, 5
    x = torch.arange(B * s * world * C, dtype=torch.float32).view(B, s, world, C) + 1000 * rank
    y = _seq_to_head(x, None)                     # [B, world*s, C]: every rank's slice of block `rank`
    back = _head_to_seq(y, None)
    return x, y, back


@pytest.mark.parametrize("world", [2, 3])
def test_all_to_all_pair_roundtrip(world):
    res = run_distributed(_roundtrip, world)
    for r, (x, y, back) in enumerate(res):
        torch.testing.assert_close(back, x)
        for src in range(world):  # chunk `src` of the gathered rows is rank src's slice, block r
            torch.testing.assert_close(y[:, src * 3:(src + 1) * 3], res[src][0][:, :, r])


def _train(rank, world, batches, packed, overrides):
    from dtg.models import build_model
    from dtg.parallel.data_parallel import DataParallel, FlatAdamW
    from dtg.parallel.ulysses import ulysses_batch

    torch.manual_seed(0)
    g = torch.distributed.group.WORLD if world > 1 else None
    model = build_model("llama-tiny-d128", device="cpu", dtype=torch.float32, sp_group=g, **overrides)
    eng = DataParallel(model, mode="ddp" if world > 1 else "single", bucket_mb=1, grad_divisor=1)
    opt = FlatAdamW(eng, lr=1e-2, eps=1e-3)
    losses = []
    for ids, pos in batches:
        pos = pos if packed else None
        opt.zero_grad()
        if world > 1:
            x, lab, p, nv = ulysses_batch(ids, rank, world, pos)
            out = model(input_ids=x, labels=lab, position_ids=p, num_valid=nv)
        else:
            out = model(input_ids=ids, labels=ids, position_ids=pos)
        eng.backward(out.loss)
        opt.step()
        losses.append(out.loss.item())
    return {n: p.detach().clone() for n, p in model.named_parameters()}, losses


def _batches():
    g = torch.Generator().manual_seed(3)
    out = []
    for _ in range(2):
        ids = torch.randint(0, 512, (2, 32), generator=g)
        # packed rows: documents of 11 / 13 / 8 and 20 / 12 tokens (positions restart at 0)
        pos = torch.cat([torch.cat([torch.arange(n) for n in (11, 13, 8)])[None],
                         torch.cat([torch.arange(n) for n in (20, 12)])[None]])
        out.append((ids, pos))
    return out


@pytest.mark.parametrize("world,packed,overrides", [
    (2, False, {}),
    (2, True, {}),
    (4, False, {}),  # 4 ranks > 2 kv heads: kv heads replicated before the exchange
    (4, True, dict(num_attention_heads=8, num_key_value_heads=4, head_dim=64)),
])
def test_llama_ulysses_training_matches_single(world, packed, overrides):
    batches = _batches()
    ref, ref_losses = _train(0, 1, batches, packed, overrides)
    res = run_distributed(_train, world, batches, packed, overrides)
    assert abs(sum(r[1][0] for r in res) - ref_losses[0]) < 1e-4 * abs(ref_losses[0])
    for r in range(world):
        for n, v in ref.items():
            torch.testing.assert_close(res[r][0][n], v, atol=3e-4, rtol=1e-3, msg=f"rank {r} {n}")


def test_ulysses_batch_slices_and_labels():
    from dtg.parallel.ulysses import ulysses_batch

    x = torch.arange(2 * 12).view(2, 12)
    ids, lab, pos, nv = ulysses_batch(x, 1, 3)
    assert nv == 2 * 11 and pos is None
    assert torch.equal(ids[0], torch.tensor([4, 5, 6, 7]))
    assert torch.equal(lab[0], torch.tensor([5, 6, 7, 8]))
    ids, lab, pos, nv = ulysses_batch(x, 2, 3, position_ids=x % 5)
    assert torch.equal(lab[1], torch.tensor([21, 22, 23, -100])) and torch.equal(pos[0], x[0, 8:] % 5)
