"""Pipeline parallelism on the gfx950 kernels: 2 stages sharing the box's GPU over gloo, 1F1B with
4 micro-batches; Llama (bf16) batch loss and every parameter gradient == the unsharded model's."""
import pytest
import torch

from _dist import run_distributed

pytestmark = pytest.mark.gpu


def _grads(rank, world):
    import dtg.ops  # noqa: F401
    from dtg.models import build_model
    from dtg.parallel.data_parallel import DataParallel
    from dtg.parallel.pipeline import OneFOneB, PipelineStage

    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    model = build_model("llama-tiny-d128", device=dev, num_hidden_layers=4)
    g = torch.Generator().manual_seed(5)
    ids = torch.randint(0, 1000, (8, 256), generator=g).to(dev)
    if world == 1:
        eng = DataParallel(model, mode="single")
        eng.backward(model(input_ids=ids, labels=ids).loss)
        a, loss = 0, None
    else:
        stage = PipelineStage(model, None)
        eng = DataParallel(model, mode="single")
        loss = OneFOneB(stage, eng, num_microbatches=4).step(ids).item()
        a = stage.layer_range[0]
    torch.cuda.synchronize()
    out = {}
    for n, p in model.named_parameters():
        if n.startswith("layers."):
            i = int(n.split(".")[1])
            n = f"layers.{a + i}" + n[len(f"layers.{i}"):]
        out[n] = p.main_grad.float().cpu()
    return loss, out


def test_pipeline_llama_gpu_matches_single(cuda):
    _, ref = _grads(0, 1)
    res = run_distributed(_grads, 2)
    assert res[0][0] == res[1][0]
    got = {}
    for _, gr in res:
        for n, v in gr.items():
            got[n] = v  # the tied embedding's grad is summed over the first/last stage on both
    assert set(got) == set(ref)
    for n, v in ref.items():
        rel = ((got[n] - v).norm() / v.norm().clamp_min(1e-12)).item()
        assert rel < 2e-2, (n, rel)
