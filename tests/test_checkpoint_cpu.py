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


def _hybrid_make():
    from dtg.models import build_model
    from dtg.parallel.data_parallel import FlatAdamW
    from dtg.parallel.fsdp import FullyShard
    from dtg.parallel.tensor_parallel import make_mesh

    torch.manual_seed(0)
    replicate, shard_group, _, _, _ = make_mesh(2)
    m = build_model("llama-tiny", device="cpu", dtype=torch.float32)
    eng = FullyShard(m, group=shard_group, replicate_group=replicate, device="cpu")
    return m, eng, FlatAdamW(eng, lr=1e-2, eps=1e-3)


def _hybrid_save_worker(rank, world, batches, d):
    from dtg.train.checkpoint import save_sharded

    m, eng, opt = _hybrid_make()
    _steps(m, eng, opt, batches[:2], rank, world)
    save_sharded(os.path.join(d, "checkpoint"), eng)
    _steps(m, eng, opt, batches[2:], rank, world)
    return eng.full_state_dict(rank0_only=False)


def _hybrid_load_worker(rank, world, batches, d):
    from dtg.train.checkpoint import load_sharded

    m, eng, opt = _hybrid_make()
    load_sharded(os.path.join(d, "checkpoint"), eng)
    assert eng.step_count == 2
    _steps(m, eng, opt, batches[2:], rank, world)
    return eng.full_state_dict(rank0_only=False)


def test_hybrid_checkpoint_written_once_and_reshards():
    """HYBRID_SHARD (2 replicas x 2-way shards): only replica 0 writes, every slice is indexed
    once, and the checkpoint resumes both as HYBRID (world 4) and as FULL_SHARD (world 2)."""
    import json

    batches = _batches(512, 4, 32, n=3)
    with tempfile.TemporaryDirectory() as d:
        cont = run_distributed(_hybrid_save_worker, 4, batches, d)[0]
        meta = json.load(open(os.path.join(d, "checkpoint", "index.json")))
        assert sorted(f["rank"] for f in meta["files"]) == [0, 1], [f["rank"] for f in meta["files"]]
        for r in (2, 3):
            assert not os.path.exists(os.path.join(d, "checkpoint", f"shard_r{r:05d}.pt"))
        again = run_distributed(_hybrid_load_worker, 4, batches, d)
        for n in cont:
            torch.testing.assert_close(again[3][n], cont[n], **TOL, msg=n)
        full = run_distributed(_load_worker, 2, "fsdp", batches, d)[0]
        for n in cont:
            torch.testing.assert_close(full[n], cont[n], **TOL, msg=n)


def test_interrupted_save_keeps_previous_checkpoint(tmp_path):
    """A crash before the commit marker leaves the previous checkpoint loadable (the partial
    .pending is discarded); a crash after it is rolled forward on the next start."""
    import json
    import shutil

    from dtg.train.checkpoint import (COMMIT, CheckpointManager, has_checkpoint, new_state,
                                      recover_checkpoint)

    m, eng, opt = _make("single")
    sched = torch.optim.lr_scheduler.CosineAnnealingLR(opt, T_max=10)
    mgr = CheckpointManager(tmp_path, eng, opt, sched, "full")
    st = new_state()
    st["global_step"] = 5
    mgr.save(st)
    assert has_checkpoint(tmp_path) and not (tmp_path / ".pending").exists()
    before = torch.load(tmp_path / "model.pt", weights_only=True)
    # crash in the middle of writing the next save: a .pending without COMMIT
    pend = tmp_path / ".pending"
    pend.mkdir()
    (pend / "model.pt").write_bytes(b"partial")
    assert recover_checkpoint(tmp_path) == "discarded"
    assert not pend.exists() and json.loads((tmp_path / "state.json").read_text())["global_step"] == 5
    after = torch.load(tmp_path / "model.pt", weights_only=True)
    assert all(torch.equal(before[k], after[k]) for k in before)
    # crash after COMMIT, half-way through the roll-forward: state.json still old, new model.pt
    # already moved, the rest still pending -> the next start finishes the move
    with torch.no_grad():
        for p in m.parameters():
            p.add_(1.0)
    st["global_step"] = 9
    staging = tmp_path / "staging"
    mgr2 = CheckpointManager(staging, eng, opt, sched, "full")
    mgr2.save(st)
    pend.mkdir()
    for name in ("optimizer.pt", "lr_scheduler.pt", "rng.pt", "state.json"):
        shutil.copy(staging / name, pend / name)
    (pend / COMMIT).write_text("ok\n")
    shutil.copy(staging / "model.pt", tmp_path / "model.pt")  # moved before the crash
    assert json.loads((tmp_path / "state.json").read_text())["global_step"] == 5
    assert recover_checkpoint(tmp_path) == "rolled-forward"
    assert json.loads((tmp_path / "state.json").read_text())["global_step"] == 9 and not pend.exists()
    assert CheckpointManager(tmp_path, eng, opt, sched, "full").load()["global_step"] == 9


@pytest.mark.parametrize("style", ["full", "dp"])
def test_every_payload_is_fsynced_before_commit(tmp_path, monkeypatch, style):
    """a durable COMMIT marker must never sit next to payload a power loss could
    truncate.  Every file of the save (model / optimizer / shards / index / lr_scheduler / rng /
    state.json) and the .pending directory are fsynced BEFORE the marker is written, and the
    experiment directory after the roll-forward's renames."""
    import os as _os

    from dtg.train.checkpoint import CheckpointManager, new_state

    events = []
    real = _os.fsync

    def spy(fd):
        events.append(_os.readlink(f"/proc/self/fd/{fd}"))
        return real(fd)

    monkeypatch.setattr(_os, "fsync", spy)
    m, eng, opt = _make("single")
    sched = torch.optim.lr_scheduler.CosineAnnealingLR(opt, T_max=10)
    st = new_state()
    st["global_step"] = 3
    CheckpointManager(tmp_path, eng, opt, sched, style).save(st)
    marker = next(i for i, e in enumerate(events) if e.endswith("/.pending/COMMIT"))
    before = set(events[:marker])
    pend = str(tmp_path / ".pending")
    payload = ["lr_scheduler.pt", "rng.pt", "state.json", "model.pt"]
    payload += ["optimizer.pt"] if style == "full" else ["checkpoint/__0_0.distcp", "checkpoint/dtg.json",
                                                          "checkpoint"]
    for rel in payload:
        assert f"{pend}/{rel}" in before, rel
    assert pend in before  # the directory entries of the payload
    assert str(tmp_path) in events[marker + 1:]  # the renames into exp_dir
    assert (tmp_path / "state.json").exists() and not (tmp_path / ".pending").exists()


def _failing_write_worker(rank, world, d, async_save):
    """Rank 1's checkpoint write fails; every rank must raise (none may wait at a barrier for a
    rank that already left), and the previous checkpoint stays published."""
    import dtg.train.checkpoint as ck
    from dtg.train.checkpoint import CheckpointManager, new_state

    m, eng, opt = _make("zero")
    sched = torch.optim.lr_scheduler.CosineAnnealingLR(opt, T_max=10)
    mgr = CheckpointManager(d, eng, opt, sched, "sharded", async_save=async_save, fmt="dtg")
    st = new_state()
    st["global_step"] = 1
    mgr.save(st)
    mgr.finalize()
    if rank == 1:
        def boom(*a, **k):
            raise OSError("disk full (injected)")

        ck.write_sharded = boom
    st["global_step"] = 2
    out = []
    try:
        mgr.save(st)
        mgr.finalize()
    except RuntimeError as e:
        out.append(str(e))
    return out


@pytest.mark.parametrize("async_save", [False, True])
def test_checkpoint_write_failure_raises_on_every_rank(tmp_path, async_save):
    import json

    res = run_distributed(_failing_write_worker, 2, str(tmp_path), async_save)
    assert res[1] == ["async checkpoint write failed" if async_save else "checkpoint write failed"]
    assert res[0] == [("async checkpoint write failed" if async_save else "checkpoint write failed") + " on another rank"]
    assert json.loads((tmp_path / "state.json").read_text())["global_step"] == 1
