"""Ulysses sequence parallelism on the gfx950 kernels: 2 ranks sharing the box's GPU over gloo,
Llama (bf16, packed rows) loss and summed parameter gradients == the unsharded model's."""
import pytest
import torch

from _dist import run_distributed

pytestmark = pytest.mark.gpu


def _batch():
    g = torch.Generator().manual_seed(5)
    ids = torch.randint(0, 1000, (2, 512), generator=g)
    pos = torch.cat([torch.cat([torch.arange(n) for n in (200, 250, 62)])[None],
                     torch.cat([torch.arange(n) for n in (512,)])[None]])
    return ids, pos


def _grads(rank, world):
    import dtg.ops  # noqa: F401
    from dtg.models import build_model
    from dtg.parallel.ulysses import ulysses_batch

    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    g = torch.distributed.group.WORLD if world > 1 else None
    model = build_model("llama-tiny-d128", device=dev, sp_group=g)
    ids, pos = (t.to(dev) for t in _batch())
    if world > 1:
        x, lab, p, nv = ulysses_batch(ids, rank, world, pos)
        out = model(input_ids=x, labels=lab, position_ids=p, num_valid=nv)
    else:
        out = model(input_ids=ids, labels=ids, position_ids=pos)
    out.loss.backward()
    torch.cuda.synchronize()
    return out.loss.item(), {n: p.grad.float().cpu() for n, p in model.named_parameters()}


def test_ulysses_llama_gpu_matches_single(cuda):
    ref_loss, ref = _grads(0, 1)
    res = run_distributed(_grads, 2)
    assert abs(sum(r[0] for r in res) - ref_loss) < 2e-2 * abs(ref_loss)
    for n, v in ref.items():
        got = res[0][1][n] + res[1][1][n]
        rel = ((got - v).norm() / v.norm().clamp_min(1e-12)).item()
        assert rel < 3e-2, (n, rel)
