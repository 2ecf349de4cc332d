"""Pretrained loading (`--init-from`, dtg.models.loading): every engine layout reads exactly the
HF safetensors values into the slices it owns -- single, ZeRO and FSDP at world 2, TP = 2, and
a pipeline stage whose local layer 0 is global layer 1.

The HF directory is written here from a random model through hf_compat.llama_to_hf (split
q/k/v and gate/up tensors, two safetensors files), so the loader's fusing, TP slicing and
row-range reads are checked against the model the files came from."""
import os
import tempfile

import pytest
import torch

import dtg  # noqa: F401

from _dist import run_distributed


def _write_hf(d, model_name):
    from safetensors.torch import save_file

    from dtg.models import build_model, resolve_config
    from dtg.models.hf_compat import llama_to_hf

    cfg = resolve_config(model_name)
    torch.manual_seed(123)
    m = build_model(cfg, device="cpu", dtype=torch.float32)
    with torch.no_grad():
        for n, p in m.named_parameters():
            if n.endswith(".bias"):
                p.normal_(0, 0.1)  # non-zero biases, so a mis-sliced bias cannot pass
    sd = m.state_dict()
    hf = llama_to_hf(sd, cfg)
    if cfg.tie_word_embeddings:
        hf.pop("lm_head.weight")  # HF tied checkpoints store the matrix once
    keys = sorted(hf)
    half = len(keys) // 2
    save_file({k: hf[k].contiguous() for k in keys[:half]}, os.path.join(d, "model-00001-of-00002.safetensors"))
    save_file({k: hf[k].contiguous() for k in keys[half:]}, os.path.join(d, "model-00002-of-00002.safetensors"))
    return {k: v.clone() for k, v in sd.items()}


def _engine(kind, model, group=None, tp_group=None):
    from dtg.parallel.data_parallel import DataParallel
    from dtg.parallel.fsdp import FullyShard

    if kind == "fsdp":
        return FullyShard(model, group=group, tp_group=tp_group, device="cpu")
    return DataParallel(model, mode=kind, group=group, tp_group=tp_group, broadcast_from_rank0=False)


def _load_worker(rank, world, kind, model_name, d):
    from dtg.models import build_model, resolve_config
    from dtg.models.loading import load_pretrained

    cfg = resolve_config(model_name)
    torch.manual_seed(rank + 7)  # different garbage on every rank: only the load may fill params
    m = build_model(cfg, device="cpu", dtype=torch.float32)
    eng = _engine(kind, m)
    load_pretrained(eng, d, cfg)
    return eng.full_state_dict(rank0_only=False)


@pytest.mark.parametrize("kind,world,model_name", [("single", 1, "llama-tiny"), ("zero", 2, "llama-tiny"),
                                                   ("fsdp", 2, "llama-tiny"), ("fsdp", 2, "llama-tiny-d128"),
                                                   ("fsdp", 2, "qwen2-tiny")])
def test_load_pretrained_engines(kind, world, model_name):
    with tempfile.TemporaryDirectory() as d:
        ref = _write_hf(d, model_name)
        if world == 1:
            res = [_load_worker(0, 1, kind, model_name, d)]
        else:
            res = run_distributed(_load_worker, world, kind, model_name, d)
    for sd in res:
        for k, v in ref.items():
            assert torch.equal(sd[k].float(), v), k


def _tp_worker(rank, world, model_name, d):
    from dtg.models import build_model, resolve_config
    from dtg.models.loading import load_pretrained
    from dtg.parallel.tensor_parallel import make_mesh

    cfg = resolve_config(model_name)
    _, tp_group, _, tp_rank, _ = make_mesh(world)
    torch.manual_seed(rank + 7)
    m = build_model(cfg, device="cpu", dtype=torch.float32, tp_group=tp_group)
    eng = _engine("single", m, tp_group=tp_group)
    load_pretrained(eng, d, cfg)
    return {k: v.detach().clone() for k, v in m.state_dict().items()}, tp_rank


@pytest.mark.parametrize("model_name", ["llama-tiny", "llama-tiny-d128", "qwen2-tiny"])
def test_load_pretrained_tp2(model_name):
    from dtg.models import resolve_config
    from dtg.parallel.tensor_parallel import unshard_state_dicts

    cfg = resolve_config(model_name)
    with tempfile.TemporaryDirectory() as d:
        ref = _write_hf(d, model_name)
        res = run_distributed(_tp_worker, 2, model_name, d)
    full = unshard_state_dicts([r[0] for r in sorted(res, key=lambda r: r[1])], cfg)
    for k, v in ref.items():
        assert torch.equal(full[k].float(), v), k


def test_load_pretrained_pipeline_stage_uses_global_layer_names():
    from dtg.models import build_model, resolve_config
    from dtg.models.loading import load_pretrained

    with tempfile.TemporaryDirectory() as d:
        ref = _write_hf(d, "llama-tiny")
        cfg = resolve_config("llama-tiny", num_hidden_layers=1)
        m = build_model(cfg, device="cpu", dtype=torch.float32)
        m._dtg_layer_offset = 1  # this stage holds global layer 1 as its local layer 0
        eng = _engine("single", m)
        load_pretrained(eng, d, cfg)
    sd = m.state_dict()
    for k in sd:
        if k.startswith("layers.0."):
            assert torch.equal(sd[k], ref["layers.1." + k[len("layers.0."):]]), k


def test_load_pretrained_missing_dir_fails():
    from dtg.models import resolve_config
    from dtg.models.loading import load_pretrained

    with tempfile.TemporaryDirectory() as d, pytest.raises(FileNotFoundError):
        load_pretrained(None, d, resolve_config("llama-tiny"))
