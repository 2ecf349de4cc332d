"""DCP as the sharded chapters' checkpoint (train/dcp_ckpt.py): a 2-D
(FSDP dp 2 x TP 2) run on 4 gloo ranks writes `checkpoint/` through torch.distributed.checkpoint
from every rank; torch's own `dcp_to_torch_save` reads it into the reference's layout (HF names,
torch AdamW state with full param_groups); it resumes bit-exactly at W = 1 / TP = 1, at W = 2 /
TP = 1 and at W = 2 / TP = 2 (every loaded parameter and moment equals the stored one); the
previous dtg-sharded-v2 format stays readable through the same manager.

Reference: /root/reference/04-fully-sharded-data-parallel/train_llm.py:121-154,249-263,
06-tensor-parallel/train_llm.py:177-190,283-295."""
import json
import os

import pytest
import torch

from _dist import run_distributed

MODEL = "llama-tiny-d128"


def _batches(vocab, n=2, rows=4, S=32):
    g = torch.Generator().manual_seed(0)
    return [torch.randint(0, vocab, (rows, S), generator=g) for _ in range(n)]


def _engine(tp, kind="fsdp"):
    from dtg.models import build_model, resolve_config
    from dtg.parallel.data_parallel import DataParallel, FlatAdamW
    from dtg.parallel.fsdp import FullyShard
    from dtg.parallel.tensor_parallel import make_mesh

    cfg = resolve_config(MODEL)
    import torch.distributed as dist

    if dist.is_initialized():
        dp_group, tp_group, dp_rank, tp_rank, dp = make_mesh(tp)
    else:
        dp_group = tp_group = None
        dp_rank, dp = 0, 1
    if kind == "fsdp":
        with torch.device("meta"):
            model = build_model(cfg, tp_group=tp_group, init=False, dtype=torch.float32)
        eng = FullyShard(model, group=dp_group, tp_group=tp_group, device="cpu", seed=0)
    else:
        torch.manual_seed(0)
        model = build_model(cfg, device="cpu", dtype=torch.float32, tp_group=tp_group)
        eng = DataParallel(model, mode="zero" if dp > 1 else "single", group=dp_group, tp_group=tp_group)
    opt = FlatAdamW(eng, lr=1e-2, eps=1e-3)
    return cfg, model, eng, opt, dp_rank, dp


def _save_2d(rank, world, d):
    from dtg.train.dcp_ckpt import save_dcp

    cfg, model, eng, opt, dp_rank, dp = _engine(2)
    for ids in _batches(cfg.vocab_size):
        per = ids.shape[0] // dp
        mine = ids[dp_rank * per:(dp_rank + 1) * per]
        opt.zero_grad()
        eng.backward(model(input_ids=mine, labels=mine).loss)
        opt.step()
    save_dcp(os.path.join(d, "checkpoint"), eng, opt, cfg, global_step=2)
    return eng.step_count


def _load_and_dump(rank, world, d, tp, kind):
    """Load the checkpoint into a (world, tp) layout; return the full parameters and moments in
    HF names (TP shards re-assembled through the same DCP chunk geometry)."""
    from dtg.train.dcp_ckpt import _chunks, load_dcp

    cfg, model, eng, opt, _, _ = _engine(tp, kind)
    meta = load_dcp(os.path.join(d, "checkpoint"), eng, cfg)
    out = {}
    for hf, hshape, offs, sizes, views in _chunks(eng, cfg):
        for k, v in views.items():
            out.setdefault(k, {}).setdefault(hf, []).append((offs, v.clone()))
    return out, eng.step_count, meta


def _assemble(dumps, key, shapes):
    full = {}
    for dump in dumps:
        for hf, chunks in dump[key].items():
            t = full.setdefault(hf, torch.full(shapes[hf], float("nan")))
            for offs, v in chunks:
                idx = tuple(slice(o, o + s) for o, s in zip(offs, v.shape))
                t[idx] = v
    return full


@pytest.mark.slow
def test_dcp_2d_checkpoint_is_torch_readable_and_resumes_bit_exact(tmp_path):
    from torch.distributed.checkpoint.format_utils import dcp_to_torch_save

    d = str(tmp_path)
    steps = run_distributed(_save_2d, 4, d)
    assert steps == [2, 2, 2, 2]
    ck = tmp_path / "checkpoint"
    assert (ck / ".metadata").exists() and (ck / "__0_0.distcp").exists() and (ck / "__3_0.distcp").exists()
    # torch's own converter, the reference's README recipe
    dcp_to_torch_save(str(ck), str(tmp_path / "full.pt"))
    sd = torch.load(tmp_path / "full.pt", weights_only=True)
    assert set(sd) == {"model", "optimizer"}
    model_sd, opt_sd = sd["model"], sd["optimizer"]
    from dtg.models import resolve_config

    cfg = resolve_config(MODEL)
    d_, nq, nkv = cfg.head_dim, cfg.num_attention_heads, cfg.num_key_value_heads
    assert model_sd["model.layers.0.self_attn.q_proj.weight"].shape == (nq * d_, cfg.hidden_size)
    assert model_sd["model.layers.0.self_attn.k_proj.weight"].shape == (nkv * d_, cfg.hidden_size)
    assert model_sd["model.layers.0.mlp.gate_proj.weight"].shape == (cfg.intermediate_size, cfg.hidden_size)
    assert model_sd["model.norm.weight"].shape == (cfg.hidden_size,)
    if cfg.tie_word_embeddings:  # an HF tied model's state dict lists both names; only one has AdamW state
        assert torch.equal(model_sd["lm_head.weight"], model_sd["model.embed_tokens.weight"])
        assert "lm_head.weight" not in opt_sd["state"]
    else:
        assert model_sd["lm_head.weight"].shape == (cfg.vocab_size, cfg.hidden_size)
    assert all(torch.isfinite(v).all() for v in model_sd.values())
    st = opt_sd["state"]["model.layers.0.mlp.down_proj.weight"]
    assert set(st) == {"exp_avg", "exp_avg_sq", "step"} and float(st["step"]) == 2.0
    (pg,) = opt_sd["param_groups"]
    assert pg["lr"] == pytest.approx(1e-2) and tuple(pg["betas"]) == (0.9, 0.999) and pg["eps"] == pytest.approx(1e-3)
    assert set(pg["params"]) == set(model_sd) - ({"lm_head.weight"} if cfg.tie_word_embeddings else set())
    shapes = {k: tuple(v.shape) for k, v in model_sd.items()}
    # resume on other layouts: every loaded element equals the stored one
    for world, tp, kind in ((1, 1, "fsdp"), (2, 1, "fsdp"), (2, 2, "fsdp"), (2, 1, "zero")):
        if world == 1:
            dumps = [_load_and_dump(0, 1, d, tp, kind)]
        else:
            dumps = run_distributed(_load_and_dump, world, d, tp, kind)
        assert all(x[1] == 2 for x in dumps) and dumps[0][2]["global_step"] == 2
        got = _assemble([x[0] for x in dumps], "p", shapes)
        m = _assemble([x[0] for x in dumps], "m", shapes)
        v2 = _assemble([x[0] for x in dumps], "v", shapes)
        for k, v in model_sd.items():
            if k not in opt_sd["state"]:  # the tied head
                continue
            assert torch.equal(got[k], v), (world, tp, kind, k)
            assert torch.equal(m[k], st_k := opt_sd["state"][k]["exp_avg"]), (world, tp, kind, k, st_k.shape)
            assert torch.equal(v2[k], opt_sd["state"][k]["exp_avg_sq"]), (world, tp, kind, k)


def _dtg_roundtrip(rank, world, d):
    from dtg.train.checkpoint import CheckpointManager, new_state

    cfg, model, eng, opt, dp_rank, dp = _engine(1)
    sched = torch.optim.lr_scheduler.CosineAnnealingLR(opt, T_max=10)
    for ids in _batches(cfg.vocab_size):
        per = ids.shape[0] // dp
        mine = ids[dp_rank * per:(dp_rank + 1) * per]
        opt.zero_grad()
        eng.backward(model(input_ids=mine, labels=mine).loss)
        opt.step()
        sched.step()
    st = new_state()
    st["global_step"] = 2
    CheckpointManager(d, eng, opt, sched, "sharded", fmt="dtg").save(st)
    before = {k: v.clone() for k, v in eng.full_state_dict(rank0_only=False).items()}
    cfg, model, eng2, opt2, _, _ = _engine(1)
    sched2 = torch.optim.lr_scheduler.CosineAnnealingLR(opt2, T_max=10)
    state = CheckpointManager(d, eng2, opt2, sched2, "sharded").load()  # default fmt reads the old format
    after = eng2.full_state_dict(rank0_only=False)
    return state["global_step"], all(torch.equal(before[k], after[k]) for k in before)


@pytest.mark.slow
def test_dtg_sharded_v2_still_loads_through_the_manager(tmp_path):
    res = run_distributed(_dtg_roundtrip, 2, str(tmp_path))
    assert (tmp_path / "checkpoint" / "index.json").exists()
    assert all(step == 2 and same for step, same in res)


def _async_save_overlapped(rank, world, d):
    """dp 2 x tp 2: two steps, an async DCP save, two more steps while the writer runs (its file
    writes held back until those steps are done), then finalize.  Returns this rank's chunks at
    the saved step and after the later steps."""
    import threading
    import time

    import dtg.train.dcp_ckpt as dc
    from dtg.train.checkpoint import CheckpointManager, new_state

    started, steps_done = threading.Event(), threading.Event()
    real = dc.write_dcp

    def held(*a, **k):  # the writer starts, then waits for the training thread's two steps
        started.set()
        steps_done.wait(60)
        return real(*a, **k)

    dc.write_dcp = held
    cfg, model, eng, opt, dp_rank, dp = _engine(2)
    sched = torch.optim.lr_scheduler.CosineAnnealingLR(opt, T_max=10)
    batches = _batches(cfg.vocab_size, n=4)

    def step(ids):
        per = ids.shape[0] // dp
        mine = ids[dp_rank * per:(dp_rank + 1) * per]
        opt.zero_grad()
        eng.backward(model(input_ids=mine, labels=mine).loss)
        opt.step()
        sched.step()

    def dump():
        return {(hf, tuple(offs)): {k: v.clone() for k, v in views.items()}
                for hf, hshape, offs, sizes, views in dc._chunks(eng, cfg)}

    for ids in batches[:2]:
        step(ids)
    saved = dump()
    mgr = CheckpointManager(d, eng, opt, sched, "sharded", async_save=True, fmt="dcp")
    st = new_state()
    st["global_step"] = 2
    t0 = time.perf_counter()
    mgr.save(st)
    stall = time.perf_counter() - t0
    assert started.wait(60)
    for ids in batches[2:]:
        step(ids)
    steps_done.set()
    later = dump()
    mgr.finalize()
    return saved, later, stall


@pytest.mark.slow
def test_async_dcp_save_overlaps_training_and_resumes_bit_exact(tmp_path):
    d = str(tmp_path)
    res = run_distributed(_async_save_overlapped, 4, d)
    ck = tmp_path / "checkpoint"
    assert (ck / ".metadata").exists() and not (tmp_path / ".pending").exists()
    assert json.loads((tmp_path / "state.json").read_text())["global_step"] == 2
    # the later steps really changed the state the writer was holding a snapshot of
    assert any(not torch.equal(res[0][0][k]["p"], res[0][1][k]["p"]) for k in res[0][0])
    from torch.distributed.checkpoint.format_utils import dcp_to_torch_save

    dcp_to_torch_save(str(ck), str(tmp_path / "full.pt"))
    sd = torch.load(tmp_path / "full.pt", weights_only=True)
    model_sd, opt_sd = sd["model"], sd["optimizer"]
    for saved, _, _ in res:  # the checkpoint holds the step-2 snapshot, not the live buffers
        for (hf, offs), views in saved.items():
            idx = tuple(slice(o, o + s) for o, s in zip(offs, views["p"].shape))
            assert torch.equal(model_sd[hf][idx], views["p"]), hf
            assert torch.equal(opt_sd["state"][hf]["exp_avg_sq"][idx], views["v"]), hf
    # and it resumes bit-exactly on another layout (W = 2, TP = 1)
    shapes = {k: tuple(v.shape) for k, v in model_sd.items()}
    dumps = run_distributed(_load_and_dump, 2, d, 1, "fsdp")
    got = _assemble([x[0] for x in dumps], "p", shapes)
    m = _assemble([x[0] for x in dumps], "m", shapes)
    for k in opt_sd["state"]:
        assert torch.equal(got[k], model_sd[k]) and torch.equal(m[k], opt_sd["state"][k]["exp_avg"]), k
