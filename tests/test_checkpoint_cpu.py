"""T4: checkpoint round trips -- sharded (FSDP/ZeRO) save on W ranks, load on W' ranks; full
single-device layout; resumed training continues like an uninterrupted run."""
import os
import tempfile

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
        assert os.path.exists(os.path.join(d, "checkpoint", ".metadata"))
        assert os.path.exists(os.path.join(d, "checkpoint", "__1_0.distcp"))
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
