"""Pipeline parallelism (1F1B over point-to-point activations) == one process: Llama trained
with 2 and 4 stages (tied and untied lm_head, stages x data-parallel replicas) reaches the
single-process parameters and losses, on gloo ranks."""
import pytest
import torch

import dtg  # noqa: F401
import dtg.ops  # noqa: F401

from _dist import run_distributed

LAYERS = 4


def _train(rank, world, pp, batches, overrides, micro):
    import torch.distributed as dist

    from dtg.models import build_model
    from dtg.parallel.data_parallel import DataParallel, FlatAdamW
    from dtg.parallel.pipeline import OneFOneB, PipelineStage
    from dtg.parallel.tensor_parallel import make_mesh

    torch.manual_seed(0)
    model = build_model("llama-tiny-d128", device="cpu", dtype=torch.float32, num_hidden_layers=LAYERS, **overrides)
    names_all = [n for n, _ in model.named_parameters()]
    if world == 1:
        eng = DataParallel(model, mode="single")
        opt = FlatAdamW(eng, lr=1e-2, eps=1e-3)
        losses = []
        for ids in batches:
            opt.zero_grad()
            out = model(input_ids=ids, labels=ids)
            eng.backward(out.loss)
            opt.step()
            losses.append(out.loss.item())
        return {n: p.detach().clone() for n, p in model.named_parameters()}, losses, None
    dp_group, pp_group, dp_rank, pp_rank, dp = make_mesh(pp)
    stage = PipelineStage(model, pp_group)
    eng = DataParallel(model, mode="ddp" if dp > 1 else "single", group=dp_group)
    opt = FlatAdamW(eng, lr=1e-2, eps=1e-3)
    sched = OneFOneB(stage, eng, num_microbatches=micro)
    losses = []
    for ids in batches:
        rows = ids.shape[0] // dp
        mine = ids[dp_rank * rows:(dp_rank + 1) * rows]
        nv = int((mine[:, 1:] != -100).sum())
        # every replica's loss is the mean over its rows; the dp average makes it the batch mean
        opt.zero_grad()
        loss = sched.step(mine, num_valid=nv)
        opt.step()
        t = loss.clone()
        if dp > 1:
            dist.all_reduce(t, group=dp_group)
            t /= dp
        losses.append(t.item())
    a, b = stage.layer_range
    rename = {}
    for n, p in model.named_parameters():
        if n.startswith("layers."):
            i = int(n.split(".")[1])
            n = "layers." + str(a + i) + n[len("layers." + str(i)):]
        rename[n] = p.detach().clone()
    return rename, losses, stage.partition


@pytest.mark.parametrize("world,pp,overrides,micro", [
    (2, 2, {}, 4),                              # tied embedding split across first/last stage
    (4, 4, {"tie_word_embeddings": False}, 4),  # one layer per stage, micro-batches = stages
    (4, 2, {}, 2),                              # 2 stages x 2 data-parallel replicas
    (3, 3, {"tie_word_embeddings": False}, 6),  # more micro-batches than stages
])
def test_llama_pipeline_matches_single(world, pp, overrides, micro):
    g = torch.Generator().manual_seed(7)
    batches = [torch.randint(0, 512, (12 if world == 3 else 8, 16), generator=g) for _ in range(2)]
    ref, ref_losses, _ = _train(0, 1, 1, batches, overrides, micro)
    res = run_distributed(_train, world, pp, batches, overrides, micro)
    for r in range(world):
        assert abs(res[r][1][0] - ref_losses[0]) < 1e-4 * abs(ref_losses[0]), (res[r][1], ref_losses)
        for n, v in res[r][0].items():
            torch.testing.assert_close(v, ref[n], atol=3e-4, rtol=1e-3, msg=f"rank {r} {n}")
    owned = set().union(*[set(r[0]) for r in res])
    assert owned == set(ref), set(ref) ^ owned


def test_balanced_partition():
    from dtg.models import resolve_config
    from dtg.parallel.pipeline import balanced_partition, head_cost_in_layers

    assert balanced_partition(8, 2) == [4, 4]
    assert balanced_partition(4, 4) == [1, 1, 1, 1]
    cfg = resolve_config("llama-3-8b")
    c = head_cost_in_layers(cfg)
    assert 2.0 < c < 3.0
    parts = balanced_partition(32, 4, c)
    assert sum(parts) == 32 and parts[-1] < parts[0]
