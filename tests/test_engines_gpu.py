"""Distributed engines driving the real gfx950 kernels: ZeRO-2 and FSDP (ZeRO-3) with two ranks
sharing the test box's one GPU (gloo carries the collectives, as RCCL refuses two ranks on one
device), against a single-process run of the same bf16 Llama on the same GPU."""
import pytest
import torch

from _dist import run_distributed

pytestmark = pytest.mark.gpu
MODEL = "llama-tiny-d128"
STEPS = 3


def _batches(vocab):
    g = torch.Generator().manual_seed(0)
    return [torch.randint(0, vocab, (4, 128), generator=g) for _ in range(STEPS)]


def _train(engine_kind, rank, world):
    from dtg.models import build_model, resolve_config
    from dtg.parallel.data_parallel import DataParallel, FlatAdamW

    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    cfg = resolve_config(MODEL)
    torch.manual_seed(0)
    model = build_model(cfg, device=dev)
    if engine_kind == "fsdp":
        from dtg.parallel.fsdp import FullyShard

        eng = FullyShard(model, device=dev)
    else:
        eng = DataParallel(model, mode=engine_kind if world > 1 else "single", bucket_mb=1)
    opt = FlatAdamW(eng, lr=1e-3)
    losses = []
    for ids in _batches(cfg.vocab_size):
        per = ids.shape[0] // world
        mine = ids[rank * per:(rank + 1) * per].to(dev)
        opt.zero_grad()
        out = model(input_ids=mine, labels=mine)
        eng.backward(out.loss)
        opt.step()
        losses.append(out.loss.item())
    if engine_kind == "fsdp":
        sd = eng.full_state_dict(rank0_only=False)
        return {k: v.float().cpu() for k, v in sd.items()}, losses
    if hasattr(eng, "wait_param_gather"):
        eng.wait_param_gather()
    torch.cuda.synchronize()
    return {n: p.detach().float().cpu() for n, p in model.named_parameters()}, losses


def _worker(rank, world, kind):
    return _train(kind, rank, world)


@pytest.mark.parametrize("kind", ["zero", "fsdp"])
def test_engine_two_ranks_one_gpu_matches_single(cuda, kind):
    ref, ref_losses = _train("single", 0, 1)
    res = run_distributed(_worker, 2, kind)
    for r in range(2):
        params, losses = res[r]
        # step 1 sees identical weights: the mean of the two half-batch losses == full-batch loss
        assert abs(sum(x[0] for x in (res[0][1], res[1][1])) / 2 - ref_losses[0]) < 2e-2 * abs(ref_losses[0])
        for n, v in ref.items():
            rel = ((params[n] - v).norm() / v.norm().clamp_min(1e-12)).item()
            assert rel < 2e-2, (kind, r, n, rel)
