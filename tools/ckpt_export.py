#!/usr/bin/env python3
"""Get a trained model out of (or into) this framework's sharded checkpoints.

A `dtg-sharded-v2` checkpoint (`{exp_dir}/checkpoint/`: index.json + shard_rNNNNN.pt, written
by FSDP / ZeRO / TP / 2-D / PP runs on any world size) is consolidated on ONE CPU process, one
parameter at a time from the memory-mapped shards, into

  * model.pt           this framework's full state dict (what chapter 01's `model.pt` holds; load
                       it with `model.load_state_dict` or `--init-from`-style tooling), and/or
  * HF safetensors     model-0000k-of-0000n.safetensors + model.safetensors.index.json +
                       config.json, via `dtg.models.hf_compat` (fused qkv / gate_up split back into
                       q/k/v and gate/up), loadable by `transformers.AutoModelForCausalLM`;
  * --with-optimizer   the AdamW moments as exp_avg.pt / exp_avg_sq.pt (full shapes);
  * DCP (--format dcp) a torch.distributed.checkpoint directory in the reference's FSDP layout
                       ({"model": HF-named tensors[, "optimizer": ...]}), for torch's own
                       `dcp_to_torch_save` / `dcp.load`.

Host memory: `hf` keeps one safetensors shard (--max-shard-gb) in memory and `dcp` spills each
parameter to memory-mapped scratch, so both stay near one parameter; `pt` / `both` (and
--with-optimizer's .pt files) hold the whole model -- 2 bytes per parameter, 3x that with the
moments -- until torch.save writes it: use `hf` or `dcp` for 70B / 405B checkpoints.

The reverse direction, `import`, turns HF safetensors, a model.pt or a DCP checkpoint into a one-shard
dtg-sharded-v2 checkpoint; the sharded loader reshards it onto any (data-parallel x tensor-
parallel) layout on resume.

    python tools/ckpt_export.py export outputs/llama-fsdp/checkpoint --model llama-3-8b --out export/ --format both
    python tools/ckpt_export.py import /weights/Meta-Llama-3-8B --model llama-3-8b --out outputs/ft/checkpoint

Reference: the reference converts DCP checkpoints with torch's format utilities
(/root/reference/04-fully-sharded-data-parallel/README.md:244-248); this is the equivalent for
this framework's own format.
"""
from __future__ import annotations

import argparse
import dataclasses
import json
import os
import sys
from pathlib import Path

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import torch  # noqa: E402

import dtg  # noqa: E402,F401
from dtg.models import resolve_config  # noqa: E402
from dtg.models.config import LlamaConfig  # noqa: E402
from dtg.train.checkpoint import iter_full_params, read_index, write_single_shard  # noqa: E402


def _hf_items(name, t, cfg):
    """This framework's (name, tensor) -> HF (name, tensor) pairs (one parameter at a time)."""
    from dtg.models.hf_compat import llama_to_hf

    if not isinstance(cfg, LlamaConfig):
        raise SystemExit("HF export supports the Llama family (llama / qwen2 / mistral) configs")
    untied = dataclasses.replace(cfg, tie_word_embeddings=False)
    return list(llama_to_hf({name: t}, untied).items())


def export(ckpt_dir, out, model=None, fmt="both", with_optimizer=False, max_shard_gb=5.0, dtype=None):
    out = Path(out)
    out.mkdir(parents=True, exist_ok=True)
    meta = read_index(ckpt_dir)
    cfg = resolve_config(model) if model else None
    if fmt in ("hf", "both") and cfg is None:
        raise SystemExit("--model is needed for the HF export (the config names the fused splits)")
    what = ("p", "m", "v") if with_optimizer else ("p",)
    cast = (lambda t: t.to(dtype)) if dtype is not None else (lambda t: t)
    model_sd, m_sd, v_sd = {}, {}, {}
    hf_files, hf_cur, hf_bytes, weight_map = [], {}, 0, {}
    limit = int(max_shard_gb * (1 << 30))

    def flush():
        nonlocal hf_cur, hf_bytes
        if hf_cur:
            from safetensors.torch import save_file

            fname = f"model-{len(hf_files) + 1:05d}.safetensors"
            save_file({k: v.contiguous() for k, v in hf_cur.items()}, str(out / fname), metadata={"format": "pt"})
            hf_files.append((fname, list(hf_cur)))
            hf_cur, hf_bytes = {}, 0

    for name, d in iter_full_params(ckpt_dir, what):
        p = cast(d["p"])
        if fmt in ("pt", "both"):
            model_sd[name] = p
        if with_optimizer:
            m_sd[name], v_sd[name] = d["m"], d["v"]
        if fmt in ("hf", "both"):
            for hn, ht in _hf_items(name, p, cfg):
                if hn == "lm_head.weight" and cfg.tie_word_embeddings:
                    continue
                nb = ht.numel() * ht.element_size()
                if hf_bytes and hf_bytes + nb > limit:
                    flush()
                hf_cur[hn] = ht.clone()
                hf_bytes += nb
    if fmt in ("hf", "both"):
        flush()
        n = len(hf_files)
        total = 0
        for i, (fname, keys) in enumerate(hf_files):
            new = f"model-{i + 1:05d}-of-{n:05d}.safetensors"
            os.replace(out / fname, out / new)
            for k in keys:
                weight_map[k] = new
        for f in out.glob("model-*-of-*.safetensors"):
            total += f.stat().st_size
        with open(out / "model.safetensors.index.json", "w") as fp:
            json.dump({"metadata": {"total_size": total}, "weight_map": weight_map}, fp, indent=1)
        from dtg.models.hf_compat import hf_llama_config

        hf_llama_config(cfg).to_json_file(str(out / "config.json"))
    if fmt in ("pt", "both"):
        torch.save(model_sd, out / "model.pt")
    if with_optimizer:
        torch.save(m_sd, out / "exp_avg.pt")
        torch.save(v_sd, out / "exp_avg_sq.pt")
    summary = {"source": str(ckpt_dir), "world_size": meta["world_size"], "tp_size": meta["tp_size"],
               "step": meta["step"], "global_step": meta.get("global_step"), "params": len(meta["param_shapes_global"]),
               "hf_files": len(hf_files)}
    with open(out / "export.json", "w") as fp:
        json.dump(summary, fp, indent=1)
    return summary


def _hf_moments(name, m, cfg):
    """Moments follow their parameter through the same fused -> HF split."""
    return dict(_hf_items(name, m, cfg))


def export_dcp(ckpt_dir, out, model, with_optimizer=False):
    """dtg-sharded-v2 -> a torch.distributed.checkpoint (DCP) directory (`.metadata` +
    `__0_0.distcp`) laid out like the reference's FSDP checkpoints
    (/root/reference/04-fully-sharded-data-parallel/train_llm.py:121-154): {"model": {HF fqn:
    tensor}} plus, with the optimizer, {"optimizer": {"state": {fqn: {step, exp_avg,
    exp_avg_sq}}, "param_groups": [...]}} -- readable by torch's own format utilities
    (`dcp_to_torch_save`, README.md:244-248) and by `dcp.load` into an HF-named model.

    Each full parameter is assembled once into a memory-mapped scratch file next to the output
    (page cache, not resident memory) and DCP writes from those views, so host RSS stays about
    one parameter even for a 405B export; the scratch is deleted afterwards."""
    import numpy as np
    import torch.distributed.checkpoint as dcp

    out = Path(out)
    out.mkdir(parents=True, exist_ok=True)
    meta = read_index(ckpt_dir)
    cfg = resolve_config(model)
    scratch = out / ".dcp_scratch"
    scratch.mkdir(exist_ok=True)
    what = ("p", "m", "v") if with_optimizer else ("p",)
    model_sd, opt_state, k = {}, {}, 0

    def spill(t):
        nonlocal k
        t = t.contiguous()
        if t.dtype == torch.bfloat16:
            view = np.memmap(scratch / f"{k}.bin", dtype=np.int16, mode="w+", shape=tuple(t.shape))
            view[...] = t.view(torch.int16).numpy()
            k += 1
            return torch.from_numpy(view).view(torch.bfloat16)
        view = np.memmap(scratch / f"{k}.bin", dtype=np.float32 if t.dtype == torch.float32 else None, mode="w+",
                         shape=tuple(t.shape))
        view[...] = t.numpy()
        k += 1
        return torch.from_numpy(view)

    for name, d in iter_full_params(ckpt_dir, what):
        hf = _hf_items(name, d["p"], cfg)
        ms = _hf_moments(name, d["m"], cfg) if with_optimizer else {}
        vs = _hf_moments(name, d["v"], cfg) if with_optimizer else {}
        for hn, ht in hf:
            if hn == "lm_head.weight" and cfg.tie_word_embeddings:
                continue
            model_sd[hn] = spill(ht)
            if with_optimizer:
                opt_state[hn] = {"step": torch.tensor(float(meta["step"])), "exp_avg": spill(ms[hn]),
                                 "exp_avg_sq": spill(vs[hn])}
    state = {"model": model_sd}
    if with_optimizer:
        # torch AdamW's full param_group (the reference resumes through get_state_dict + dcp.load +
        # set_state_dict, 04-fully-sharded-data-parallel/train_llm.py:133-146); lr from the run's
        # lr_scheduler.pt next to checkpoint/ when present
        from dtg.train.dcp_ckpt import _adamw_group

        group = _adamw_group(None)
        sched = Path(ckpt_dir).parent / "lr_scheduler.pt"
        if sched.exists():
            last = torch.load(sched, weights_only=True).get("_last_lr")
            if last:
                group["lr"] = float(last[0])
        state["optimizer"] = {"state": opt_state, "param_groups": [dict(group, params=list(opt_state))]}
    dcp.save(state, checkpoint_id=str(out), no_dist=True)
    import shutil

    del model_sd, opt_state, state
    shutil.rmtree(scratch, ignore_errors=True)
    summary = {"source": str(ckpt_dir), "format": "dcp", "world_size": meta["world_size"], "tp_size": meta["tp_size"],
               "step": meta["step"], "global_step": meta.get("global_step"), "params": len(meta["param_shapes_global"])}
    with open(out / "export.json", "w") as fp:
        json.dump(summary, fp, indent=1)
    return summary


def import_dcp(src, out, model, step=0):
    """A DCP checkpoint with an HF-named {"model": ...} (the reference's FSDP layout, or
    export_dcp's) -> a one-shard dtg-sharded-v2 checkpoint (moments too when the DCP holds an
    "optimizer" entry).  Goes through torch's own `dcp_to_torch_save` (weights-only tensors) and
    loads the result with `torch.load(weights_only=True)`."""
    import tempfile

    from torch.distributed.checkpoint.format_utils import dcp_to_torch_save

    from dtg.models.hf_compat import llama_from_hf

    cfg = resolve_config(model)
    with tempfile.TemporaryDirectory(dir=str(Path(out).parent) if Path(out).parent.exists() else None) as tmp:
        path = os.path.join(tmp, "full.pt")
        dcp_to_torch_save(str(src), path)
        sd = torch.load(path, map_location="cpu", weights_only=True)
    hf = sd["model"] if "model" in sd else sd
    hf = {k: v for k, v in hf.items() if not (k == "lm_head.weight" and cfg.tie_word_embeddings)}
    params = llama_from_hf(hf, cfg)
    moments = None
    if "optimizer" in sd and sd["optimizer"].get("state"):
        st = sd["optimizer"]["state"]
        m = llama_from_hf({k: st[k]["exp_avg"] for k in hf}, cfg)
        v = llama_from_hf({k: st[k]["exp_avg_sq"] for k in hf}, cfg)
        moments = {n: (m[n], v[n]) for n in params}
        step = int(float(next(iter(st.values()))["step"]))
    return write_single_shard(out, params, moments, step=step)


def import_(src, out, model, step=0):
    """HF safetensors directory / file, or a model.pt of this framework -> one-shard checkpoint."""
    from dtg.models.hf_compat import llama_from_hf

    src = Path(src)
    cfg = resolve_config(model)
    if src.suffix == ".pt":
        sd = torch.load(src, map_location="cpu", weights_only=True)
    else:
        from safetensors.torch import load_file

        files = sorted(src.glob("*.safetensors")) if src.is_dir() else [src]
        hf = {}
        for f in files:
            hf.update(load_file(str(f)))
        if cfg.tie_word_embeddings:
            hf.pop("lm_head.weight", None)
        sd = llama_from_hf(hf, cfg)
    return write_single_shard(out, sd, step=step)


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    sub = ap.add_subparsers(dest="cmd", required=True)
    e = sub.add_parser("export")
    e.add_argument("ckpt_dir", help="a dtg-sharded-v2 checkpoint/ directory")
    e.add_argument("--out", required=True)
    e.add_argument("--model", default=None, help="bundled config name or HF config dir (needed for --format hf)")
    e.add_argument("--format", default="both", choices=["pt", "hf", "both", "dcp"],
                   help="pt / both hold the whole model (and with --with-optimizer its moments) in host memory "
                        "until written; hf streams safetensors shards; dcp streams through memory-mapped scratch")
    e.add_argument("--with-optimizer", action="store_true")
    e.add_argument("--max-shard-gb", type=float, default=5.0)
    e.add_argument("--dtype", default=None, choices=[None, "bf16", "fp32"])
    i = sub.add_parser("import")
    i.add_argument("src", help="HF safetensors dir/file, a model.pt, or a DCP checkpoint directory (.metadata)")
    i.add_argument("--model", required=True)
    i.add_argument("--out", required=True, help="checkpoint/ directory to create")
    a = ap.parse_args(argv)
    if a.cmd == "export":
        if a.format == "dcp":
            if a.model is None:
                raise SystemExit("--model is needed for the DCP export (HF names)")
            print(json.dumps(export_dcp(a.ckpt_dir, a.out, a.model, a.with_optimizer)))
            return
        dt = {"bf16": torch.bfloat16, "fp32": torch.float32}.get(a.dtype)
        print(json.dumps(export(a.ckpt_dir, a.out, a.model, a.format, a.with_optimizer, a.max_shard_gb, dt)))
    else:
        if (Path(a.src) / ".metadata").exists():
            meta = import_dcp(a.src, a.out, a.model)
        else:
            meta = import_(a.src, a.out, a.model)
        print(json.dumps({"out": a.out, "params": len(meta["param_shapes_global"])}))


if __name__ == "__main__":
    main()
