"""Sharded-checkpoint export / import (tools/ckpt_export.py): a 2-D (FSDP W=2 x TP=2) checkpoint
becomes a model.pt equal to the trained parameters and HF safetensors whose transformers model
gives the same logits; the reverse import resumes on a different layout."""
import os
import sys
import tempfile

import torch

import dtg  # noqa: F401

from _dist import run_distributed
from test_engines_cpu import _batches

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
MODEL = "llama-tiny-d128"


def _save_2d(rank, world, batches, d):
    from dtg.models import build_model, resolve_config
    from dtg.parallel.data_parallel import FlatAdamW
    from dtg.parallel.fsdp import FullyShard
    from dtg.parallel.tensor_parallel import make_mesh, shard_full_state_dict
    from dtg.train.checkpoint import save_sharded

    dp_group, tp_group, dp_rank, tp_rank, dp = make_mesh(2)
    cfg = resolve_config(MODEL)
    torch.manual_seed(0)
    full = build_model(cfg, device="cpu", dtype=torch.float32)
    model = build_model(cfg, device="cpu", dtype=torch.float32, tp_group=tp_group, init=False)
    model.load_state_dict(shard_full_state_dict(full.state_dict(), cfg, tp_rank, 2))
    eng = FullyShard(model, group=dp_group, tp_group=tp_group, device="cpu")
    opt = FlatAdamW(eng, lr=1e-2, eps=1e-3)
    for ids in batches:
        per = ids.shape[0] // dp
        mine = ids[dp_rank * per:(dp_rank + 1) * per]
        opt.zero_grad()
        out = model(input_ids=mine, labels=mine)
        eng.backward(out.loss)
        opt.step()
    save_sharded(os.path.join(d, "checkpoint"), eng)
    return eng.full_state_dict(rank0_only=False), tp_rank


def _load_tp2(rank, world, d):
    from dtg.models import build_model, resolve_config
    from dtg.parallel.data_parallel import DataParallel
    from dtg.parallel.tensor_parallel import make_mesh
    from dtg.train.checkpoint import load_sharded

    _, tp_group, _, tp_rank, _ = make_mesh(2)
    cfg = resolve_config(MODEL)
    model = build_model(cfg, device="cpu", dtype=torch.float32, tp_group=tp_group, init=False)
    eng = DataParallel(model, mode="single", tp_group=tp_group, broadcast_from_rank0=False)
    load_sharded(d, eng)
    return {n: p.detach().clone() for n, p in model.named_parameters()}, tp_rank


def test_export_2d_checkpoint_to_pt_and_hf_then_import():
    import ckpt_export
    from transformers import AutoModelForCausalLM

    from dtg.models import build_model, resolve_config
    from dtg.parallel.tensor_parallel import unshard_state_dicts

    cfg = resolve_config(MODEL)
    batches = _batches(cfg.vocab_size, 4, 32, n=2)
    with tempfile.TemporaryDirectory() as d:
        res = run_distributed(_save_2d, 4, batches, d)
        by_tp = {tp: sd for sd, tp in res}
        trained = unshard_state_dicts([by_tp[0], by_tp[1]], cfg)
        out = os.path.join(d, "export")
        summary = ckpt_export.export(os.path.join(d, "checkpoint"), out, model=MODEL, fmt="both", max_shard_gb=0.0005)
        assert summary["world_size"] == 4 and summary["tp_size"] == 2 and summary["hf_files"] > 1
        sd = torch.load(os.path.join(out, "model.pt"), weights_only=True)
        assert set(sd) == set(trained)
        for n, v in trained.items():
            assert torch.equal(sd[n], v), n
        # HF safetensors -> transformers: same logits as this framework's model with model.pt
        ours = build_model(cfg, device="cpu", dtype=torch.float32)
        ours.load_state_dict(sd)
        hf = AutoModelForCausalLM.from_pretrained(out, torch_dtype=torch.float32)
        ids = batches[0][:2]
        a = ours(input_ids=ids, labels=ids, return_logits=True)
        b = hf(input_ids=ids, labels=ids)
        torch.testing.assert_close(a.logits, b.logits, atol=1e-4, rtol=1e-4)
        # reverse: HF dir -> one-shard checkpoint -> resumes on a TP=2 layout
        ck2 = os.path.join(d, "imported")
        ckpt_export.import_(out, ck2, MODEL)
        res2 = run_distributed(_load_tp2, 2, ck2)
        back = unshard_state_dicts([r[0] for r in sorted(res2, key=lambda r: r[1])], cfg)
        for n, v in trained.items():
            assert torch.equal(back[n], v), n


def test_export_rejects_incomplete_checkpoint(tmp_path):
    import pytest

    from dtg.train.checkpoint import iter_full_params, write_single_shard

    write_single_shard(tmp_path, {"w": torch.ones(4, 3), "b": torch.zeros(3)})
    got = dict(iter_full_params(tmp_path))
    assert got["w"]["p"].shape == (4, 3) and got["b"]["p"].shape == (3,)
    import json

    meta = json.loads((tmp_path / "index.json").read_text())
    meta["files"][0]["index"][0][2][0][1] = 2  # the stored rectangle now covers 2 of 4 rows
    (tmp_path / "index.json").write_text(json.dumps(meta))
    with pytest.raises(RuntimeError, match="covered"):
        dict(iter_full_params(tmp_path))


def test_dcp_export_readable_by_torch_format_utils_and_imports_back():
    """a 2-D (FSDP W=2 x TP=2) checkpoint exported as a torch DCP directory is
    read by torch's own `dcp_to_torch_save` into the reference's {"model", "optimizer"} layout
    with HF names (same values as the trained model, moments included), and imports back onto a
    TP=2 layout bit-exactly."""
    import ckpt_export
    from torch.distributed.checkpoint.format_utils import dcp_to_torch_save

    from dtg.models import resolve_config
    from dtg.models.hf_compat import llama_to_hf
    from dtg.parallel.tensor_parallel import unshard_state_dicts

    cfg = resolve_config(MODEL)
    batches = _batches(cfg.vocab_size, 4, 32, n=2)
    with tempfile.TemporaryDirectory() as d:
        res = run_distributed(_save_2d, 4, batches, d)
        by_tp = {tp: sd for sd, tp in res}
        trained = unshard_state_dicts([by_tp[0], by_tp[1]], cfg)
        out = os.path.join(d, "dcp")
        s = ckpt_export.export_dcp(os.path.join(d, "checkpoint"), out, MODEL, with_optimizer=True)
        assert s["format"] == "dcp" and os.path.exists(os.path.join(out, ".metadata"))
        assert not os.path.exists(os.path.join(out, ".dcp_scratch"))
        dcp_to_torch_save(out, os.path.join(d, "full.pt"))
        sd = torch.load(os.path.join(d, "full.pt"), weights_only=True)
        want = llama_to_hf(trained, cfg)
        assert set(sd["model"]) == {k for k in want if not (k == "lm_head.weight" and cfg.tie_word_embeddings)}
        for k, v in sd["model"].items():
            assert torch.equal(v, want[k]), k
        st = sd["optimizer"]["state"]
        assert set(st) == set(sd["model"]) and all(float(x["step"]) == 2 for x in st.values())
        assert all(x["exp_avg"].shape == sd["model"][k].shape for k, x in st.items())
        (pg,) = sd["optimizer"]["param_groups"]  # torch AdamW's full group
        assert {"lr", "betas", "eps", "weight_decay"} <= set(pg) and set(pg["params"]) == set(st)
        # DCP -> one-shard checkpoint -> TP=2 resume, bit-exact parameters
        ck2 = os.path.join(d, "imported")
        ckpt_export.import_dcp(out, ck2, MODEL)
        res2 = run_distributed(_load_tp2, 2, ck2)
        back = unshard_state_dicts([r[0] for r in sorted(res2, key=lambda r: r[1])], cfg)
        for n, v in trained.items():
            assert torch.equal(back[n], v), n
