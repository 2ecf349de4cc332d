"""--async-ckpt with the reference's DCP tree on the GPU: FSDP on 2 ranks sharing the box's GPU
(gloo between them).  The save snapshots the engine's HBM-resident parameter shards and moments
into pinned host buffers (non-blocking copies, one device sync), the writer thread runs DCP over
its own gloo group while two more training steps change the device state, and the published
checkpoint holds the saved step's values bit for bit (train/dcp_ckpt.py HostPool / write_dcp,
train/checkpoint.py CheckpointManager)."""
import json
import os

import pytest
import torch

from _dist import run_distributed

pytestmark = pytest.mark.gpu
MODEL = "llama-tiny-d128"


def _worker(rank, world, d, device="cuda:0"):
    import threading

    import torch.distributed as dist

    import dtg.train.dcp_ckpt as dc
    from dtg.models import build_model, resolve_config
    from dtg.parallel.data_parallel import FlatAdamW
    from dtg.parallel.fsdp import FullyShard
    from dtg.train.checkpoint import CheckpointManager, new_state

    dev = torch.device(device)
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    steps_done = threading.Event()
    real = dc.write_dcp

    def held(*a, **k):  # the writer waits for the training thread's two later steps
        steps_done.wait(120)
        return real(*a, **k)

    dc.write_dcp = held
    cfg = resolve_config(MODEL)
    with torch.device("meta"):
        model = build_model(cfg, init=False)
    eng = FullyShard(model, group=dist.group.WORLD, device=dev, seed=0)
    opt = FlatAdamW(eng, lr=1e-3)
    sched = torch.optim.lr_scheduler.CosineAnnealingLR(opt, T_max=10)
    g = torch.Generator().manual_seed(0)
    batches = [torch.randint(0, cfg.vocab_size, (4, 64), generator=g) for _ in range(4)]

    def step(ids):
        mine = ids[rank * 2:(rank + 1) * 2].to(dev)
        opt.zero_grad()
        eng.backward(model(input_ids=mine, labels=mine).loss)
        opt.step()
        sched.step()

    def dump():
        if dev.type == "cuda":
            torch.cuda.synchronize()
        return {(hf, tuple(offs)): {k: v.detach().float().cpu() for k, v in views.items()}
                for hf, hshape, offs, sizes, views in dc._chunks(eng, cfg)}

    for ids in batches[:2]:
        step(ids)
    saved = dump()
    mgr = CheckpointManager(d, eng, opt, sched, "sharded", async_save=True, fmt="dcp")
    st = new_state()
    st["global_step"] = 2
    mgr.save(st)
    for ids in batches[2:]:
        step(ids)
    later = dump()
    steps_done.set()
    mgr.finalize()
    return saved, later


def test_async_dcp_snapshot_of_hbm_state_is_the_saved_step(cuda, tmp_path):
    from torch.distributed.checkpoint.format_utils import dcp_to_torch_save

    res = run_distributed(_worker, 2, str(tmp_path))
    assert json.loads((tmp_path / "state.json").read_text())["global_step"] == 2
    assert any(not torch.equal(res[0][0][k]["p"], res[0][1][k]["p"]) for k in res[0][0])
    dcp_to_torch_save(str(tmp_path / "checkpoint"), str(tmp_path / "full.pt"))
    sd = torch.load(tmp_path / "full.pt", weights_only=True)
    for saved, _ in res:
        for (hf, offs), views in saved.items():
            idx = tuple(slice(o, o + s) for o, s in zip(offs, views["p"].shape))
            assert torch.equal(sd["model"][hf][idx].float(), views["p"]), hf
            assert torch.equal(sd["optimizer"]["state"][hf]["exp_avg"][idx].float(), views["m"]), hf
            assert torch.equal(sd["optimizer"]["state"][hf]["exp_avg_sq"][idx].float(), views["v"]), hf
