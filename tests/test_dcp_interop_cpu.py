"""Interop of this framework's DCP checkpoints with the reference's own resume code, both ways
(ADVICE r5 dcp_ckpt.py:285).

(a) This trainer's engines write `checkpoint/` (save_dcp); the reference's resume path --
    `get_state_dict(model, optimizer, StateDictOptions(full_state_dict=False, cpu_offload=True))`
    -> `dcp.load(dict(model=..., optimizer=...))` -> `set_state_dict` on an HF `*ForCausalLM` with
    `torch.optim.AdamW(fused=True)` and a `CosineAnnealingLR` -- loads it, and every parameter and
    both AdamW moments are bit-equal to the engine's, `step` and `param_groups` survive.
(b) The reference's save (`dcp.save(dict(model=..., optimizer=...))` of the same state dicts)
    resumes in this framework's engines (load_dcp) on W = 1 and on W = 2 FSDP, bit-equal.

Reference: /root/reference/04-fully-sharded-data-parallel/train_llm.py:113-147 (resume),
:249-263 (save)."""
import os

import pytest
import torch

from _dist import run_distributed

T_MAX, LR = 1000, 3e-3


def _ids(vocab, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.randint(0, vocab, (4, 32), generator=g)


def _ours(model_name, tp=1, kind="single"):
    import torch.distributed as dist

    from dtg.models import build_model, resolve_config
    from dtg.parallel.data_parallel import DataParallel, FlatAdamW
    from dtg.parallel.fsdp import FullyShard

    cfg = resolve_config(model_name)
    group = dist.group.WORLD if dist.is_initialized() else None
    if kind == "fsdp":
        with torch.device("meta"):
            model = build_model(cfg, init=False, dtype=torch.bfloat16)
        eng = FullyShard(model, group=group, device="cpu", seed=0)
    else:
        torch.manual_seed(0)
        model = build_model(cfg, device="cpu", dtype=torch.bfloat16)
        eng = DataParallel(model, mode=kind, group=group)
    opt = FlatAdamW(eng, lr=LR, eps=1e-8, weight_decay=0.01)
    sched = torch.optim.lr_scheduler.CosineAnnealingLR(opt, T_max=T_MAX, eta_min=LR * 1e-2)
    return cfg, model, eng, opt, sched


def _hf(cfg):
    from dtg.models.hf_compat import hf_causal_lm_class, hf_llama_config

    torch.manual_seed(1)
    m = hf_causal_lm_class(cfg)(hf_llama_config(cfg)).to(torch.bfloat16)  # the reference trains bf16
    opt = torch.optim.AdamW(m.parameters(), lr=LR, fused=True)
    sched = torch.optim.lr_scheduler.CosineAnnealingLR(opt, T_max=T_MAX, eta_min=LR * 1e-2)
    return m, opt, sched


def _opts():
    from torch.distributed.checkpoint.state_dict import StateDictOptions

    return StateDictOptions(full_state_dict=False, cpu_offload=True)


def _engine_full(eng, cfg):
    """{hf name: {"p", "m", "v"}} of the engine's state, this rank's chunks (offsets attached)."""
    from dtg.train.dcp_ckpt import _chunks

    out = {}
    for hf, hshape, offs, sizes, views in _chunks(eng, cfg):
        out.setdefault(hf, []).append((hshape, offs, {k: v.detach().clone() for k, v in views.items()}))
    return out


def _assemble(dumps):
    full = {}
    for dump in dumps:
        for hf, pieces in dump.items():
            for hshape, offs, views in pieces:
                slot = full.setdefault(hf, {k: torch.full(hshape, float("nan"), dtype=v.dtype) for k, v in views.items()})
                idx = tuple(slice(o, o + s) for o, s in zip(offs, views["p"].shape))
                for k, v in views.items():
                    slot[k][idx] = v
    return full


def _train_and_save(rank, world, d, model_name, kind):
    from dtg.train.dcp_ckpt import save_dcp

    cfg, model, eng, opt, sched = _ours(model_name, kind=kind)
    for s in range(2):
        ids = _ids(cfg.vocab_size, s)
        per = ids.shape[0] // world
        mine = ids[rank * per:(rank + 1) * per]
        opt.zero_grad()
        eng.backward(model(input_ids=mine, labels=mine).loss)
        opt.step()
        sched.step()
    save_dcp(os.path.join(d, "checkpoint"), eng, opt, cfg, global_step=2)
    return _engine_full(eng, cfg)


def _reference_resume(d, cfg):
    """The reference's resume block, verbatim in behaviour (04-fully-sharded-data-parallel/
    train_llm.py:132-147) on a single process."""
    import torch.distributed.checkpoint as dcp
    from torch.distributed.checkpoint.state_dict import get_state_dict, set_state_dict

    m, opt, sched = _hf(cfg)
    msd, osd = get_state_dict(m, opt, options=_opts())
    dcp.load(dict(model=msd, optimizer=osd), checkpoint_id=os.path.join(d, "checkpoint"))
    set_state_dict(m, opt, model_state_dict=msd, optim_state_dict=osd, options=_opts())
    return m, opt


@pytest.mark.parametrize("model_name,world,kind", [("llama-tiny", 1, "single"), ("qwen2-tiny", 1, "single"),
                                                   ("llama-tiny-d128", 2, "fsdp"), ("llama-tiny", 2, "zero")])
def test_reference_resume_loads_our_checkpoint(tmp_path, model_name, world, kind):
    from dtg.models import resolve_config

    d = str(tmp_path)
    if world == 1:
        dumps = [_train_and_save(0, 1, d, model_name, kind)]
    else:
        dumps = run_distributed(_train_and_save, world, d, model_name, kind)
    ours = _assemble(dumps)
    cfg = resolve_config(model_name)
    m, opt = _reference_resume(d, cfg)
    params = dict(m.named_parameters())
    assert set(params) - {"lm_head.weight"} <= set(ours)
    osd = opt.state_dict()
    names = osd["param_groups"][0]["params"]  # indices, in named_parameters() order of the optimizer
    by_name = dict(zip([n for n, _ in m.named_parameters()], names))
    for n, p in params.items():
        src = ours["model.embed_tokens.weight" if (n == "lm_head.weight" and cfg.tie_word_embeddings) else n]
        assert torch.equal(p.detach(), src["p"]), n
        st = osd["state"][by_name[n]]
        assert torch.equal(st["exp_avg"], src["m"]), n
        assert torch.equal(st["exp_avg_sq"], src["v"]), n
        assert float(st["step"]) == 2.0
    (pg,) = osd["param_groups"]
    assert pg["lr"] == pytest.approx(LR * 1e-2 + (LR - LR * 1e-2) * (1 + torch.cos(torch.tensor(2 * torch.pi / T_MAX)).item()) / 2)
    assert pg["initial_lr"] == pytest.approx(LR) and tuple(pg["betas"]) == (0.9, 0.999)
    assert pg["weight_decay"] == pytest.approx(0.01)


def _reference_save(d, cfg):
    """The reference's training step + save block (train_llm.py:249-263) on an HF model."""
    import torch.distributed.checkpoint as dcp
    from torch.distributed.checkpoint.state_dict import get_state_dict

    m, opt, sched = _hf(cfg)
    for s in range(2):
        ids = _ids(cfg.vocab_size, s)
        opt.zero_grad()
        m(input_ids=ids, labels=ids).loss.backward()
        opt.step()
        sched.step()
    msd, osd = get_state_dict(m, opt, options=_opts())
    dcp.save(dict(model=msd, optimizer=osd), checkpoint_id=os.path.join(d, "checkpoint"))
    state = opt.state_dict()
    order = [n for n, _ in m.named_parameters()]
    return ({n: p.detach().clone() for n, p in m.named_parameters()},
            {order[i]: {k: v.clone() for k, v in s.items()} for i, s in state["state"].items()})


def _our_resume(rank, world, d, model_name, kind):
    from dtg.train.dcp_ckpt import load_dcp

    cfg, model, eng, opt, sched = _ours(model_name, kind=kind)
    load_dcp(os.path.join(d, "checkpoint"), eng, cfg)
    return _engine_full(eng, cfg), eng.step_count


@pytest.mark.parametrize("model_name,world,kind", [("llama-tiny", 1, "single"), ("qwen2-tiny", 1, "single"),
                                                   ("llama-tiny-d128", 2, "fsdp")])
def test_reference_checkpoint_resumes_in_our_engines(tmp_path, model_name, world, kind):
    from dtg.models import resolve_config

    d = str(tmp_path)
    cfg = resolve_config(model_name)
    params, state = _reference_save(d, cfg)
    if world == 1:
        res = [_our_resume(0, 1, d, model_name, kind)]
    else:
        res = run_distributed(_our_resume, world, d, model_name, kind)
    assert all(step == 2 for _, step in res)
    ours = _assemble([x for x, _ in res])
    for n, p in params.items():
        if n == "lm_head.weight" and cfg.tie_word_embeddings:
            continue
        assert torch.equal(ours[n]["p"], p), n
        assert torch.equal(ours[n]["m"], state[n]["exp_avg"]), n
        assert torch.equal(ours[n]["v"], state[n]["exp_avg_sq"]), n
