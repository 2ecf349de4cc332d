"""T3: sharding plans with no hardware -- the FSDP layout under a fake process group (W = 64)
matches the planner, and the Llama-3.1-405B plan at W = 64..512 has the sizes SURVEY §7.5 /
BASELINE.md derive (8 B/param pure-bf16 state, 6.4 GB per-layer gather, fits 288 GB at W >= 16)."""
import pytest
import torch
import torch.distributed as dist

import dtg  # noqa: F401


@pytest.fixture
def fake_pg():
    from torch.testing._internal.distributed.fake_pg import FakeStore

    dist.init_process_group("fake", store=FakeStore(), rank=3, world_size=64)
    try:
        yield
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("policy,min_params", [("transformer", 0), ("size", 20_000)])
def test_fsdp_engine_layout_matches_plan_under_fake_pg(fake_pg, policy, min_params):
    from dtg.models import build_model
    from dtg.parallel.data_parallel import FlatAdamW
    from dtg.parallel.fsdp import FullyShard
    from dtg.parallel.plan import fsdp_plan

    model = build_model("llama-tiny", device="meta", dtype=torch.float32, init=False)
    plan = fsdp_plan(model, 64, policy, min_params)
    eng = FullyShard(model, policy=policy, min_num_params=min_params, device="cpu")
    assert (eng.world, eng.rank) == (64, 3)
    assert [u.shard_numel for u in eng.units] == [u.shard_numel for u in plan.units]
    assert eng.root.shard_numel == plan.root.shard_numel
    assert eng.shard_params.numel() == plan.shard_numel
    # one full step runs end to end on no-op collectives (plumbing only: values are not real)
    opt = FlatAdamW(eng, lr=1e-3)
    ids = torch.randint(0, 256, (2, 16))
    opt.zero_grad()
    out = model(input_ids=ids, labels=ids)
    eng.backward(out.loss)
    opt.step()


@pytest.mark.parametrize("world", [64, 128, 256, 512])
def test_llama405b_fsdp_plan(world):
    from dtg.models import build_model, resolve_config
    from dtg.parallel.plan import fsdp_plan

    cfg = resolve_config("llama-3.1-405b")
    model = build_model(cfg, device="meta", init=False)
    plan = fsdp_plan(model, world)
    assert len(plan.units) == cfg.num_hidden_layers == 126
    assert plan.total_params == cfg.num_params()
    assert abs(plan.total_params / 1e9 - 405.85) < 0.01
    H, I, d = cfg.hidden_size, cfg.intermediate_size, cfg.head_dim
    layer = H * (cfg.num_attention_heads + 2 * cfg.num_key_value_heads) * d + cfg.num_attention_heads * d * H + 3 * H * I + 2 * H
    assert all(u.numel == layer for u in plan.units)
    assert abs(plan.largest_gather_bytes() / 1e9 - 6.375) < 0.01  # per-layer all-gather
    assert plan.padding_fraction() < 1e-4
    per_rank = plan.per_rank_state_bytes() / 1e9
    assert abs(per_rank - 8 * 405.85 / world) < 0.05


def test_llama405b_memory_fit_matches_survey():
    """8 GPUs cannot hold the pure-bf16 405B state (406 GB/GPU); 16 can (203 GB/GPU)."""
    from dtg.models import build_model
    from dtg.parallel.plan import fsdp_plan

    model = build_model("llama-3.1-405b", device="meta", init=False)
    p8, p16 = fsdp_plan(model, 8), fsdp_plan(model, 16)
    assert p8.per_rank_state_bytes() / 1e9 > 288
    assert p16.per_rank_state_bytes() / 1e9 + 2 * p16.largest_gather_bytes() / 1e9 < 288 * 0.92
