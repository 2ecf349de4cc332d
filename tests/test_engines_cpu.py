"""T2: data-parallel engines on gloo (world 2) reproduce a single-process run on the full batch."""
import pytest
import torch

import dtg  # noqa: F401

from _dist import run_distributed

STEPS = 3


def _batches(vocab, B, S, n=STEPS, seed=0):
    g = torch.Generator().manual_seed(seed)
    return [torch.randint(0, vocab, (B, S), generator=g) for _ in range(n)]


def _train(model_name, mode, rank, world, batches, bucket_mb=1, accum=1, overlap=False):
    from dtg.models import build_model
    from dtg.parallel.data_parallel import DataParallel, FlatAdamW

    torch.manual_seed(0)
    model = build_model(model_name, device="cpu", dtype=torch.float32)
    eng = DataParallel(model, mode=mode, bucket_mb=bucket_mb, overlap_optimizer=overlap)
    opt = FlatAdamW(eng, lr=1e-2, eps=1e-3)  # eps >> float reduction-order noise (Adam amplifies it)
    losses = []
    for ids in batches:
        per = ids.shape[0] // world
        mine = ids[rank * per:(rank + 1) * per]
        opt.zero_grad()
        micro = mine.chunk(accum)
        for i, mb in enumerate(micro):
            if i < accum - 1:
                with eng.no_sync():
                    out = model(input_ids=mb, labels=mb)
                    eng.backward(out.loss)
            else:
                out = model(input_ids=mb, labels=mb)
                eng.backward(out.loss)
        opt.step()
        losses.append(out.loss.item())
    if hasattr(eng, "wait_param_gather"):
        eng.wait_param_gather()  # ZeRO leaves the last all-gather in flight until the next forward
    return {n: p.detach().clone() for n, p in model.named_parameters()}, losses


def _worker(rank, world, model_name, mode, batches, accum, overlap=False):
    return _train(model_name, mode, rank, world, batches, accum=accum, overlap=overlap)


@pytest.mark.parametrize("model_name", ["llama-tiny", "gpt2-tiny"])
@pytest.mark.parametrize("mode", ["ddp", "zero"])
def test_data_parallel_matches_single(model_name, mode):
    batches = _batches(512, 4, 32)
    ref, _ = _train(model_name, "single", 0, 1, batches)
    res = run_distributed(_worker, 2, model_name, mode, batches, 1)
    for r in range(2):
        params, _ = res[r]
        for n in ref:
            torch.testing.assert_close(params[n], ref[n], atol=3e-4, rtol=1e-3, msg=f"rank {r} {n}")


@pytest.mark.parametrize("world", [4, 8])
def test_zero_wide_world_matches_single(world):
    """The bench's N=4 / N=8 layout: every bucket split 4 or 8 ways (padded tails, ranks whose
    slice of a small bucket is all padding), one sequence per rank."""
    batches = _batches(512, 8, 16)
    ref, _ = _train("llama-tiny", "single", 0, 1, batches)
    res = run_distributed(_worker, world, "llama-tiny", "zero", batches, 1)
    for r in (0, world - 1):
        for n in ref:
            torch.testing.assert_close(res[r][0][n], ref[n], atol=3e-4, rtol=1e-3, msg=f"rank {r} {n}")


def test_ddp_gradient_accumulation_no_sync():
    """2 ranks x 2 micro-batches with no_sync == 1 process on the full batch."""
    batches = _batches(512, 8, 16)
    ref, _ = _train("llama-tiny", "single", 0, 1, batches)
    res = run_distributed(_worker, 2, "llama-tiny", "ddp", batches, 2)
    for n in ref:
        torch.testing.assert_close(res[0][0][n], ref[n], atol=3e-4, rtol=1e-3, msg=n)


def test_flat_buffers_are_views_and_buckets_cover_params():
    from dtg.models import build_model
    from dtg.parallel.data_parallel import DataParallel

    m = build_model("llama-tiny", device="cpu", dtype=torch.float32)
    n_before = sum(p.numel() for p in m.parameters())
    eng = DataParallel(m, mode="single", bucket_mb=1)
    buf = eng.space.param_buf
    for p in m.parameters():
        assert p.untyped_storage().data_ptr() == buf.untyped_storage().data_ptr()
        assert p.main_grad.untyped_storage().data_ptr() == eng.space.grad_buf.untyped_storage().data_ptr()
        assert p.data_ptr() % 16 == 0
    assert sum(p.numel() for p in m.parameters()) == n_before
    assert len(eng.space.buckets) > 1
    assert eng.space.buckets[-1].end == eng.space.numel


@pytest.mark.parametrize("model_name", ["llama-tiny", "gpt2-tiny"])
def test_optimizer_in_backward_single_is_exact(model_name):
    """overlap_optimizer (per-bucket AdamW during backward) == the post-backward step, bit for bit."""
    batches = _batches(512, 4, 32)
    ref, lr = _train(model_name, "single", 0, 1, batches)
    got, lg = _train(model_name, "single", 0, 1, batches, overlap=True)
    assert lr == lg
    for n in ref:
        assert torch.equal(got[n], ref[n]), n


@pytest.mark.parametrize("mode,accum", [("ddp", 1), ("zero", 1), ("zero", 2)])
def test_optimizer_in_backward_distributed(mode, accum):
    batches = _batches(512, 8, 16)
    ref, _ = _train("llama-tiny", "single", 0, 1, batches)
    res = run_distributed(_worker, 2, "llama-tiny", mode, batches, accum, True)
    for r in range(2):
        for n in ref:
            torch.testing.assert_close(res[r][0][n], ref[n], atol=3e-4, rtol=1e-3, msg=f"rank {r} {n}")
