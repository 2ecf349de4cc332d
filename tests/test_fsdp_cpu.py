"""T2/T3: the FSDP (ZeRO-3) engine on gloo reproduces single-process training; policies,
meta-device init, activation checkpointing and CPU offload."""
import pytest
import torch

import dtg  # noqa: F401

from _dist import run_distributed
from test_engines_cpu import _batches, _train

TOL = dict(atol=3e-4, rtol=1e-3)


def _fsdp_train(rank, world, model_name, batches, policy, min_params, reshard, ac, offload):
    from dtg.models import build_model
    from dtg.parallel.data_parallel import FlatAdamW
    from dtg.parallel.fsdp import FullyShard
    from dtg.parallel.checkpointing import apply_activation_checkpointing

    torch.manual_seed(0)
    model = build_model(model_name, device="cpu", dtype=torch.float32)
    if ac:
        apply_activation_checkpointing(model)
    eng = FullyShard(model, policy=policy, min_num_params=min_params, reshard_after_forward=reshard,
                     cpu_offload=offload, device="cpu")
    opt = FlatAdamW(eng, lr=1e-2, eps=1e-3)
    for ids in batches:
        per = ids.shape[0] // world
        mine = ids[rank * per:(rank + 1) * per]
        opt.zero_grad()
        out = model(input_ids=mine, labels=mine)
        eng.backward(out.loss)
        opt.step()
    sd = eng.full_state_dict(rank0_only=False)
    return sd, len(eng.units)


@pytest.mark.parametrize("model_name,policy,min_params,reshard,ac", [
    ("llama-tiny", "transformer", 0, True, False),
    ("llama-tiny", "size", 100_000, True, False),
    ("llama-tiny", "transformer", 0, False, True),
    ("gpt2-tiny", "transformer", 0, True, True),
])
def test_fsdp_matches_single(model_name, policy, min_params, reshard, ac):
    batches = _batches(512, 4, 32)
    ref, _ = _train(model_name, "single", 0, 1, batches)
    res = run_distributed(_fsdp_train, 2, model_name, batches, policy, min_params, reshard, ac, False)
    for r in range(2):
        sd, nunits = res[r]
        assert nunits >= 1
        for n in ref:
            torch.testing.assert_close(sd[n], ref[n], **TOL, msg=f"rank {r} {n}")


def test_fsdp_world1_cpu_offload_and_meta_init():
    from dtg.models import build_model
    from dtg.parallel.data_parallel import FlatAdamW
    from dtg.parallel.fsdp import FullyShard

    batches = _batches(512, 2, 16)
    ref, _ = _train("llama-tiny", "single", 0, 1, batches)
    sd, _ = _fsdp_train(0, 1, "llama-tiny", batches, "transformer", 0, True, False, True)
    for n in ref:
        torch.testing.assert_close(sd[n], ref[n], **TOL, msg=n)
    # meta-device construction: only shards are materialised, init is seeded per unit
    with torch.device("meta"):
        m = build_model("llama-tiny", dtype=torch.float32, init=False)
    eng = FullyShard(m, device="cpu")
    opt = FlatAdamW(eng, lr=1e-3)
    ids = batches[0]
    out = m(input_ids=ids, labels=ids)
    eng.backward(out.loss)
    opt.step()
    assert torch.isfinite(out.loss) and abs(out.loss.item() - 6.24) < 0.5
    full = eng.full_state_dict()
    assert torch.allclose(full["layers.0.input_layernorm.weight"], torch.ones(256), atol=1e-2)
    assert full["layers.0.self_attn.qkv_proj.weight"].std().item() == pytest.approx(0.02, rel=0.1)


def test_size_policy_units():
    from dtg.models import build_model
    from dtg.parallel.fsdp import size_based_units, transformer_units

    m = build_model("llama-tiny", device="meta", dtype=torch.float32, init=False)
    assert len(transformer_units(m)) == m.config.num_hidden_layers
    units = size_based_units(m, 100_000)
    # mlp (393k) and self_attn (196k) exceed the threshold in every layer; Weight holders never
    # become units (they are not called, so they could not be gathered by hooks)
    assert len(units) == 2 * m.config.num_hidden_layers
    assert all(not getattr(u, "_dtg_param_holder", False) for u in units)


def _hybrid_train(rank, world, model_name, batches, shard, accum=1, offload=False):
    import torch.distributed as dist

    from dtg.models import build_model
    from dtg.parallel.data_parallel import FlatAdamW
    from dtg.parallel.fsdp import FullyShard
    from dtg.parallel.tensor_parallel import make_mesh

    torch.manual_seed(0)
    replicate, shard_group, _, _, n_rep = make_mesh(shard)
    model = build_model(model_name, device="cpu", dtype=torch.float32)
    eng = FullyShard(model, group=shard_group, replicate_group=replicate, device="cpu", cpu_offload=offload)
    opt = FlatAdamW(eng, lr=1e-2, eps=1e-3)
    n_rep_ar = [0]
    real = dist.all_reduce

    def counting(t, *a, group=None, **kw):
        if group is replicate:
            n_rep_ar[0] += 1
        return real(t, *a, group=group, **kw)

    dist.all_reduce = counting
    try:
        for ids in batches:
            per = ids.shape[0] // world
            mine = ids[rank * per:(rank + 1) * per]
            opt.zero_grad()
            for j, mb in enumerate(mine.chunk(accum)):
                if j < accum - 1:
                    with eng.no_sync():
                        eng.backward(model(input_ids=mb, labels=mb).loss)
                else:
                    eng.backward(model(input_ids=mb, labels=mb).loss)
            opt.step()
    finally:
        dist.all_reduce = real
    return eng.full_state_dict(rank0_only=False), eng.mode, eng.world, eng.replicas, n_rep_ar[0], len(eng.all_units)


def test_hybrid_shard_matches_single():
    """HYBRID_SHARD: 2 replicas x 2-way shards (world 4) reproduce single-process training."""
    batches = _batches(512, 4, 32)
    ref, _ = _train("llama-tiny", "single", 0, 1, batches)
    res = run_distributed(_hybrid_train, 4, "llama-tiny", batches, 2)
    for r in range(4):
        sd, mode, w, reps, _, _ = res[r]
        assert (mode, w, reps) == ("hybrid", 2, 2)
        for n in ref:
            torch.testing.assert_close(sd[n], ref[n], **TOL, msg=f"rank {r} {n}")


@pytest.mark.parametrize("offload", [False, True])
def test_hybrid_shard_accumulation_one_replica_allreduce_per_step(offload):
    """with 2 accumulated micro-batches the inter-replica all-reduce runs once per
    unit per optimizer step (on the final micro-batch, over the accumulated shard), not once per
    micro-batch -- and the result still equals single-process training on the full batch."""
    batches = _batches(512, 8, 16)
    ref, _ = _train("llama-tiny", "single", 0, 1, batches)
    res = run_distributed(_hybrid_train, 4, "llama-tiny", batches, 2, 2, offload)
    for r in range(4):
        sd, mode, _, _, n_ar, n_units = res[r]
        assert mode == "hybrid" and n_ar == n_units * len(batches), (n_ar, n_units)
        for n in ref:
            torch.testing.assert_close(sd[n], ref[n], **TOL, msg=f"rank {r} {n}")


def _offload_train(rank, world, batches, overlap, accum, offload=True, offload_params=True, ring=0):
    from dtg.models import build_model
    from dtg.parallel.data_parallel import FlatAdamW
    from dtg.parallel.fsdp import FullyShard

    torch.manual_seed(0)
    model = build_model("llama-tiny", device="cpu", dtype=torch.float32)
    eng = FullyShard(model, cpu_offload=offload, device="cpu", overlap_cpu_step=overlap,
                     offload_params=offload_params, grad_ring=ring)
    opt = FlatAdamW(eng, lr=1e-2, eps=1e-3)
    sched = torch.optim.lr_scheduler.LambdaLR(opt, lambda s: 1.0 / (1 + s))  # lr changes every step
    stepped_in_bwd = []
    for ids in batches:
        per = ids.shape[0] // world
        mine = ids[rank * per:(rank + 1) * per]
        opt.zero_grad()
        micro = mine.chunk(accum)
        for j, mb in enumerate(micro):
            ctx = eng.no_sync() if j < accum - 1 else torch.enable_grad()
            with ctx:
                eng.backward(model(input_ids=mb, labels=mb).loss)
        stepped_in_bwd.append(eng._bwd_stepped)
        opt.step()
        sched.step()
    return eng.full_state_dict(rank0_only=False), stepped_in_bwd


@pytest.mark.parametrize("accum", [1, 2])
def test_fsdp_offload_overlapped_host_step_is_bit_identical(accum):
    """overlap_cpu_step: host AdamW per unit during the last micro-batch's backward gives exactly
    the post-backward update (world 2, changing lr, with and without gradient accumulation)."""
    batches = _batches(512, 4, 32, n=3)  # 2 rows per rank -> accum micro-batches of 1 row
    on = run_distributed(_offload_train, 2, batches, True, accum)
    off = run_distributed(_offload_train, 2, batches, False, accum)
    for r in range(2):
        assert all(on[r][1]) and not any(off[r][1])
        for n, t in off[r][0].items():
            assert torch.equal(on[r][0][n], t), f"rank {r} {n}"


@pytest.mark.parametrize("overlap,accum", [(True, 1), (False, 2), (True, 2)])
def test_fsdp_resident_param_offload_is_bit_identical(overlap, accum):
    """offload_params=False (ZeRO-Offload layout: parameter shard resident in device memory,
    gradients + AdamW on the host, updated shards copied back) == the full offload."""
    batches = _batches(512, 4, 32, n=3)
    res = run_distributed(_offload_train, 2, batches, overlap, accum, True, False)
    full = run_distributed(_offload_train, 2, batches, overlap, accum, True, True)
    for r in range(2):
        for n, t in full[r][0].items():
            assert torch.equal(res[r][0][n], t), f"rank {r} {n}"


@pytest.mark.parametrize("offload", [False, True])
def test_fsdp_grad_accumulation_matches_full_batch(offload):
    """Two micro-batches (first under no_sync) == one full batch: every micro-batch's fresh full
    gradient is overwritten, not accumulated into (regression: uninitialised memory was summed)."""
    batches = _batches(512, 4, 32, n=2)
    one = run_distributed(_offload_train, 2, batches, False, 1, offload)
    two = run_distributed(_offload_train, 2, batches, False, 2, offload)
    for n, t in one[0][0].items():
        torch.testing.assert_close(two[0][0][n], t, **TOL, msg=n)  # pre-fix error: ~2 x lr = 2e-2


def test_fsdp_overlapped_host_step_guards_misuse():
    """with overlap_cpu_step the update runs inside the final backward, so (a) a second
    backward without step()/no_sync() must raise instead of updating twice, (b) step() with
    hyper-parameters that differ from the ones the in-backward update used must raise, and
    (c) last_microbatch=False accumulates with no host update."""
    from dtg.models import build_model
    from dtg.parallel.data_parallel import FlatAdamW
    from dtg.parallel.fsdp import FullyShard

    torch.manual_seed(0)
    model = build_model("llama-tiny", device="cpu", dtype=torch.float32)
    eng = FullyShard(model, cpu_offload=True, device="cpu", overlap_cpu_step=True)
    opt = FlatAdamW(eng, lr=1e-2, eps=1e-3)
    ids = torch.randint(0, 512, (2, 16), generator=torch.Generator().manual_seed(0))
    opt.zero_grad()
    eng.backward(model(input_ids=ids, labels=ids).loss)
    assert eng._bwd_stepped
    with pytest.raises(RuntimeError, match="already applied"):
        eng.backward(model(input_ids=ids, labels=ids).loss)
    opt.param_groups[0]["lr"] = 5e-3
    with pytest.raises(RuntimeError, match="different hyper-parameters"):
        opt.step()
    opt.param_groups[0]["lr"] = 1e-2
    opt.step()
    assert eng.step_count == 1 and not eng._bwd_stepped
    opt.zero_grad()
    before = eng.shard_params.clone()
    eng.backward(model(input_ids=ids, labels=ids).loss, last_microbatch=False)
    assert not eng._bwd_stepped and torch.equal(before, eng.shard_params)
    eng.backward(model(input_ids=ids, labels=ids).loss)  # final micro-batch: overlapped update
    assert eng._bwd_stepped and not torch.equal(before, eng.shard_params)
    opt.step()
    assert eng.step_count == 2


def test_offload_stats_account_host_update():
    """CPU offload accounting the 405B runs report: host AdamW seconds and GB/s per step over the
    log window (14 B per parameter), reset on read.  (D2H / H2D rows need a GPU.)"""
    from dtg.models import build_model
    from dtg.parallel.data_parallel import FlatAdamW
    from dtg.parallel.fsdp import FullyShard

    m = build_model("llama-tiny", device="cpu", dtype=torch.float32)
    eng = FullyShard(m, device="cpu", cpu_offload=True)
    opt = FlatAdamW(eng, lr=1e-3)
    ids = _batches(512, 2, 16)[0]
    for _ in range(2):
        opt.zero_grad()
        eng.backward(m(input_ids=ids, labels=ids).loss)
        opt.step()
    st = eng.offload_stats()
    assert st["host_adamw_s"] > 0 and st["host_adamw_gbs"] > 0
    assert "d2h_gb" not in st  # no device copies on a CPU engine
    assert eng.offload_stats() == {}  # reset after the read


@pytest.mark.parametrize("offload_params,ring", [(True, 2), (False, 1), (False, 3)])
def test_fsdp_offload_grad_ring_bit_identical(offload_params, ring):
    """The host gradient ring (no whole-model host gradient shard; each unit's gradient staged
    in one of `ring` slots the host AdamW consumes) == the full host gradient shard, bit for
    bit; one slot forces every unit to wait for the previous unit's host update."""
    batches = _batches(512, 4, 32, n=3)
    full = run_distributed(_offload_train, 2, batches, True, 1, True, offload_params, 0)
    got = run_distributed(_offload_train, 2, batches, True, 1, True, offload_params, ring)
    for r in range(2):
        assert all(got[r][1])
        for n, t in full[r][0].items():
            assert torch.equal(got[r][0][n], t), f"rank {r} {n}"


def test_fsdp_offload_grad_ring_refuses_accumulation():
    from dtg.models import build_model
    from dtg.parallel.data_parallel import FlatAdamW
    from dtg.parallel.fsdp import FullyShard

    model = build_model("llama-tiny", device="cpu", dtype=torch.float32)
    eng = FullyShard(model, cpu_offload=True, device="cpu", grad_ring=2)
    assert eng.shard_grads.numel() == 0 and len(eng._ring) == 2
    FlatAdamW(eng, lr=1e-3)
    ids = _batches(512, 2, 16)[0]
    with pytest.raises(RuntimeError, match="gradient ring"):
        with eng.no_sync():
            eng.backward(model(input_ids=ids, labels=ids).loss)
