"""T4: checkpoint round trips -- sharded (FSDP/ZeRO) save on W ranks, load on W' ranks; full
single-device layout; resumed training continues like an uninterrupted run."""
import os
import tempfile

import pytest
import torch

import dtg  # noqa: F401

from _dist import run_distributed
from test_engines_cpu import _batches

TOL = dict(atol=3e-4, rtol=1e-3)


def _make(engine_kind, model_name="llama-tiny"):
    from dtg.models import build_model
    from dtg.parallel.data_parallel import DataParallel, FlatAdamW
    from dtg.parallel.fsdp import FullyShard

    torch.manual_seed(0)
    m = build_model(model_name, device="cpu", dtype=torch.float32)
    if engine_kind == "fsdp":
        eng = FullyShard(m, device="cpu")
    else:
        eng = DataParallel(m, mode=engine_kind)
    opt = FlatAdamW(eng, lr=1e-2, eps=1e-3)
    return m, eng, opt


def _steps(m, eng, opt, batches, rank, world):
    for ids in batches:
        per = ids.shape[0] // world
        mine = ids[rank * per:(rank + 1) * per]
        opt.zero_grad()
        out = m(input_ids=mine, labels=mine)
        eng.backward(out.loss)
        opt.step()


def _save_worker(rank, world, kind, batches, d):
    from dtg.train.checkpoint import save_sharded

    m, eng, opt = _make(kind)
    _steps(m, eng, opt, batches[:2], rank, world)
    save_sharded(os.path.join(d, "checkpoint"), eng)
    _steps(m, eng, opt, batches[2:], rank, world)  # uninterrupted continuation
    return eng.full_state_dict(rank0_only=False)


def _load_worker(rank, world, kind, batches, d):
    from dtg.train.checkpoint import load_sharded

    m, eng, opt = _make(kind)
    load_sharded(os.path.join(d, "checkpoint"), eng)
    assert eng.step_count == 2
    _steps(m, eng, opt, batches[2:], rank, world)
    return eng.full_state_dict(rank0_only=False)


def test_fsdp_reshard_w2_to_w1_and_zero_w2():
    batches = _batches(512, 4, 32, n=3)
    with tempfile.TemporaryDirectory() as d:
        cont = run_distributed(_save_worker, 2, "fsdp", batches, d)[0]
        assert os.path.exists(os.path.join(d, "checkpoint", "index.json"))
        assert os.path.exists(os.path.join(d, "checkpoint", "shard_r00001.pt"))
        resumed_w1 = _load_worker(0, 1, "fsdp", batches, d)
        for n in cont:
            torch.testing.assert_close(resumed_w1[n], cont[n], **TOL, msg=n)
        resumed_zero = run_distributed(_load_worker, 2, "zero", batches, d)[1]
        for n in cont:
            torch.testing.assert_close(resumed_zero[n], cont[n], **TOL, msg=n)


def test_full_layout_manager_roundtrip():
    from dtg.train.checkpoint import CheckpointManager

    batches = _batches(512, 2, 16, n=3)
    with tempfile.TemporaryDirectory() as d:
        m, eng, opt = _make("single")
        sched = torch.optim.lr_scheduler.CosineAnnealingLR(opt, T_max=1000, eta_min=1e-4)
        _steps(m, eng, opt, batches[:2], 0, 1)
        sched.step(); sched.step()
        state = {"epoch": 0, "global_step": 2, "epoch_step": 2, "running_loss": 0.5}
        mgr = CheckpointManager(d, eng, opt, sched, "full")
        mgr.save(state)
        for f in ("model.pt", "optimizer.pt", "lr_scheduler.pt", "state.json", "rng.pt"):
            assert os.path.exists(os.path.join(d, f)), f
        _steps(m, eng, opt, batches[2:], 0, 1)
        cont = {n: p.detach().clone() for n, p in m.named_parameters()}
        m2, eng2, opt2 = _make("single")
        sched2 = torch.optim.lr_scheduler.CosineAnnealingLR(opt2, T_max=1000, eta_min=1e-4)
        st = CheckpointManager(d, eng2, opt2, sched2, "full").load()
        assert st == state and sched2.last_epoch == 2 and eng2.step_count == 2
        _steps(m2, eng2, opt2, batches[2:], 0, 1)
        for n, p in m2.named_parameters():
            torch.testing.assert_close(p.detach(), cont[n], atol=1e-6, rtol=1e-6, msg=n)


def _tp_model(rank, world, tp):
    """Llama-tiny on (world // tp) x tp ranks: TP inside, FSDP across (chapter 07's layout);
    tp == 1 is plain FSDP."""
    from dtg.models import build_model
    from dtg.parallel.data_parallel import FlatAdamW
    from dtg.parallel.fsdp import FullyShard
    from dtg.parallel.tensor_parallel import make_mesh

    torch.manual_seed(0)
    tp_group = dp_group = None
    if tp > 1:
        dp_group, tp_group, _, _, _ = make_mesh(tp)
    m = build_model("llama-tiny", device="cpu", dtype=torch.float32, tp_group=tp_group)
    eng = FullyShard(m, group=dp_group, tp_group=tp_group, device="cpu")
    opt = FlatAdamW(eng, lr=1e-2, eps=1e-3)
    return m, eng, opt


def _tp_full(eng, cfg, tp):
    """Global (un-TP) parameters and moments gathered over the TP group: (params, exp_avg sums)."""
    import torch.distributed as dist

    from dtg.parallel.tensor_parallel import unshard_state_dicts

    sd = eng.full_state_dict(rank0_only=False)
    if tp > 1:
        parts = [None] * tp
        dist.all_gather_object(parts, sd)
        sd = unshard_state_dicts(parts, cfg)
    return sd


def _tp_save_worker(rank, world, tp, batches, d):
    from dtg.train.checkpoint import save_sharded

    m, eng, opt = _tp_model(rank, world, tp)
    dp = world // tp
    _steps(m, eng, opt, batches[:2], rank // tp, dp)
    save_sharded(os.path.join(d, "checkpoint"), eng)
    return _tp_full(eng, m.config, tp)


def _tp_load_worker(rank, world, tp, batches, d):
    from dtg.train.checkpoint import load_sharded

    m, eng, opt = _tp_model(rank, world, tp)
    load_sharded(os.path.join(d, "checkpoint"), eng)
    assert eng.step_count == 2
    before = _tp_full(eng, m.config, tp)
    dp = world // tp
    _steps(m, eng, opt, batches[2:], rank // tp, dp)  # the optimizer state must be usable too
    return before, _tp_full(eng, m.config, tp)


@pytest.mark.parametrize("save_tp,load_tp", [(2, 1), (1, 2)])
def test_sharded_checkpoint_tp_reshard(save_tp, load_tp):
    """Save at TP=a, load at TP=b (2 ranks): parameters identical after load, and one more
    step from the loaded state matches one more step of an (a)-run restored at (a)."""
    batches = _batches(512, 4, 32, n=3)
    with tempfile.TemporaryDirectory() as d:
        saved = run_distributed(_tp_save_worker, save_tp if save_tp > 1 else 1, save_tp, batches, d)[0]
        world = load_tp
        got = run_distributed(_tp_load_worker, world, load_tp, batches, d)
        for n, t in saved.items():
            assert torch.equal(got[0][0][n], t), n
        same = run_distributed(_tp_load_worker, save_tp, save_tp, batches, d)
        for n, t in same[0][1].items():
            torch.testing.assert_close(got[0][1][n], t, **TOL, msg=n)


def test_sharded_checkpoint_rejects_incomplete():
    """A checkpoint whose index lost a slice (or a shard file) must fail to load, not leave
    parameters silently at their init values."""
    import json

    from dtg.train.checkpoint import load_sharded, save_sharded

    batches = _batches(512, 2, 16, n=1)
    with tempfile.TemporaryDirectory() as d:
        m, eng, opt = _make("fsdp")
        _steps(m, eng, opt, batches, 0, 1)
        ck = os.path.join(d, "checkpoint")
        save_sharded(ck, eng)
        meta = json.load(open(os.path.join(ck, "index.json")))
        meta["files"][0]["index"].pop(3)
        json.dump(meta, open(os.path.join(ck, "index.json"), "w"))
        m2, eng2, _ = _make("fsdp")
        with pytest.raises(RuntimeError, match="covers"):
            load_sharded(ck, eng2)
        os.remove(os.path.join(ck, "shard_r00000.pt"))
        with pytest.raises(FileNotFoundError):
            load_sharded(ck, eng2)
