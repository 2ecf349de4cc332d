"""Checkpoint / resume.

Directory layout under `{save_dir}/{experiment_name}/` follows the reference per chapter:
  * full (01, rime):  model.pt, optimizer.pt, lr_scheduler.pt, state.json, rng.pt
  * dp   (02):        model.pt (rank 0), lr_scheduler.pt, state.json, rng.pt + the optimizer
                      state as a sharded `checkpoint/` (the reference never saved it and then
                      crashed on resume)
  * sharded (04-07):  checkpoint/ (torch DCP: .metadata + __<rank>_0.distcp, the reference's tree;
                      train/dcp_ckpt.py), lr_scheduler.pt, state.json, rng.pt

`--ckpt-format dtg` keeps this framework's previous sharded format, which every load still reads:
format `dtg-sharded-v2` (this framework's own; not torch DCP, whose file names it does
not borrow): every rank writes `checkpoint/shard_rNNNNN.pt` holding, for each parameter slice it
owns, the parameter values and both AdamW moments (plain tensors: loadable with
`torch.load(weights_only=True)`), and rank 0 writes `checkpoint/index.json` with every slice's
position in GLOBAL parameter coordinates.  On load each rank copies the overlap of every stored
slice with the slices it owns now, so a checkpoint written on (W data-parallel x a tensor-
parallel) ranks loads on (W' x b) -- FSDP, ZeRO and DDP layouts alike -- and a load that would
leave any owned element unwritten fails.  Barriers bracket every save (reference C2) so no rank
reads a half-written directory.
"""
from __future__ import annotations

import json
import os
import random
from pathlib import Path

import numpy as np
import torch
import torch.distributed as dist

from ..utils.dist import barrier, get_rank, get_world_size

STATE_KEYS = ("epoch", "global_step", "epoch_step", "running_loss")


def new_state():
    return {"epoch": 0, "global_step": 0, "epoch_step": 0, "running_loss": 0}


def has_checkpoint(exp_dir) -> bool:
    return (Path(exp_dir) / "state.json").exists()


# ------------------------------------------------------------------------------ journal
# Every save is written whole into `{exp_dir}/.pending/` (state.json included) while the previous
# checkpoint stays untouched.  Once every rank's files are on disk rank 0 drops a COMMIT marker
# into .pending and rolls it forward: each item replaces its counterpart in exp_dir, state.json
# last, then .pending is removed.  A crash before COMMIT leaves the old checkpoint intact (the
# partial .pending is discarded on the next start); a crash after it is finished by
# `recover_checkpoint` on the next start.  Either way a launch never sees new weights beside an
# old state.json, and never loses the last complete checkpoint.
PENDING = ".pending"
COMMIT = "COMMIT"
# Durability (host crash / power loss, not just a dead process): every payload file is fsynced
# by its writer, every directory whose entries changed is fsynced, and the COMMIT marker is
# written only after all of that -- so a durable COMMIT always sits next to complete payload,
# and the roll-forward may delete the old copy.


def fsync_file(path) -> None:
    fd = os.open(path, os.O_RDONLY)
    try:
        os.fsync(fd)
    finally:
        os.close(fd)


def fsync_dir(path) -> None:
    """Make the directory's entries (creations, renames) durable."""
    fd = os.open(path, os.O_RDONLY | getattr(os, "O_DIRECTORY", 0))
    try:
        os.fsync(fd)
    finally:
        os.close(fd)


def save_durable(obj, path) -> None:
    """torch.save + fsync of the file."""
    torch.save(obj, path)
    fsync_file(path)


def _roll_forward(exp_dir: Path):
    import shutil

    pend = exp_dir / PENDING
    items = [it for it in pend.iterdir() if it.name not in (COMMIT, "state.json")]
    for item in items:
        dst = exp_dir / item.name
        if dst.is_dir():
            shutil.rmtree(dst)
        os.replace(item, dst)
    fsync_dir(exp_dir)  # the new payload's entries are durable before state.json points at them
    if (pend / "state.json").exists():
        os.replace(pend / "state.json", exp_dir / "state.json")
        fsync_dir(exp_dir)
    shutil.rmtree(pend, ignore_errors=True)


def commit_pending(exp_dir):
    """Rank 0, after every rank finished writing (and fsyncing) into .pending: publish it
    atomically."""
    exp_dir = Path(exp_dir)
    pend = exp_dir / PENDING
    for sub in [pend] + [d for d in pend.iterdir() if d.is_dir()]:
        fsync_dir(sub)  # every payload entry is durable before the marker exists
    marker = pend / COMMIT
    with open(marker, "w") as fp:
        fp.write("ok\n")
        fp.flush()
        os.fsync(fp.fileno())
    fsync_dir(pend)
    _roll_forward(exp_dir)


def recover_checkpoint(exp_dir) -> str:
    """Finish or discard an interrupted save (call on rank 0 before `has_checkpoint`, then
    barrier).  Returns "rolled-forward", "discarded" or "clean"."""
    import shutil

    exp_dir = Path(exp_dir)
    pend = exp_dir / PENDING
    if not pend.exists():
        return "clean"
    if (pend / COMMIT).exists():
        _roll_forward(exp_dir)
        return "rolled-forward"
    shutil.rmtree(pend, ignore_errors=True)
    return "discarded"


# ------------------------------------------------------------------------------ RNG (G7)
def rng_state(device):
    st = {"python": random.getstate(), "numpy": np.random.get_state(), "torch": torch.get_rng_state()}
    if torch.cuda.is_available():
        st["cuda"] = torch.cuda.get_rng_state_all()
    return st


def save_rng(path):
    st = rng_state(None)
    obj = {"python": repr(st["python"]), "numpy_keys": torch.from_numpy(st["numpy"][1].astype(np.int64)),
           "numpy_pos": st["numpy"][2], "torch": st["torch"],
           "cuda": torch.stack(st["cuda"]) if "cuda" in st else torch.empty(0)}
    if isinstance(path, _RngBox):
        path.obj = obj
    else:
        torch.save(obj, path)


class _RngBox:
    """save_rng target that keeps the state object in memory (async checkpoints)."""
    obj = None


def _to_cpu(obj):
    if torch.is_tensor(obj):
        return obj.detach().to("cpu", copy=True)
    if isinstance(obj, dict):
        return {k: _to_cpu(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_to_cpu(v) for v in obj)
    return obj


def load_rng(path, local_rank: int = 0):
    st = torch.load(path, weights_only=True)
    import ast

    random.setstate(ast.literal_eval(st["python"]))
    np.random.set_state(("MT19937", st["numpy_keys"].numpy().astype(np.uint32), int(st["numpy_pos"]), 0, 0.0))
    torch.set_rng_state(st["torch"])
    if torch.cuda.is_available() and st["cuda"].numel() > 0:
        cuda = list(st["cuda"])
        if local_rank < len(cuda):
            torch.cuda.set_rng_state(cuda[local_rank])


# ------------------------------------------------------------------------------ sharded
# Every stored slice is described in GLOBAL (un-tensor-parallel) parameter coordinates: a
# rank's TP-local flat range is cut into rectangles (global row 0, rows, global col 0, cols,
# offset in the slice's flat data).  Loading intersects the rectangles a rank owns NOW (its own
# TP degree and data-parallel sharding) with the stored ones, so one checkpoint loads on any
# (dp, tp) layout: W -> W' data-parallel ranks and TP a -> TP b, including TP -> no TP
# (reference: DCP over DTensor modules reshards on load, 06-tensor-parallel/train_llm.py:177-190,
# 283-295).  Every owned element must be covered exactly, or the load fails.
FORMAT = "dtg-sharded-v2"
INDEX = "index.json"


def _shard_file(rank: int) -> str:
    return f"shard_r{rank:05d}.pt"


def param_kind(name: str) -> str:
    """How the tensor-parallel plan (parallel/tensor_parallel.py) splits a Llama parameter."""
    if name.endswith("self_attn.qkv_proj.weight") or name.endswith("self_attn.qkv_proj.bias"):
        return "qkv"
    if name.endswith("mlp.gate_up_proj.weight"):
        return "gate_up"
    if name.endswith("self_attn.o_proj.weight") or name.endswith("mlp.down_proj.weight"):
        return "col"
    if name in ("embed_tokens.weight", "lm_head.weight"):
        return "row"
    return "rep"


class _TPGeom:
    def __init__(self, engine):
        tp = getattr(engine.module, "tp", None)
        self.rank, self.size = (tp.rank, tp.size) if tp is not None and tp.enabled else (0, 1)
        cfg = getattr(engine.module, "config", None)
        self.cfg = cfg

    def blocks(self, kind, rows_local):
        """[(local row start, rows, global row start)] of the row-sharded blocks of a param."""
        r, n = self.rank, self.size
        if kind == "qkv" and n > 1:
            d, nq, nkv = self.cfg.head_dim, self.cfg.num_attention_heads, self.cfg.num_key_value_heads
            sizes_l = [nq // n * d, nkv // n * d, nkv // n * d]
            gstart = [0, nq * d, (nq + nkv) * d]
        elif kind == "gate_up" and n > 1:
            sizes_l = [rows_local // 2, rows_local // 2]
            gstart = [0, rows_local // 2 * n]
        elif kind in ("row", "qkv", "gate_up") and n > 1:
            sizes_l, gstart = [rows_local], [0]
        else:
            return [(0, rows_local, 0)]
        out, lo = [], 0
        for sz, g in zip(sizes_l, gstart):
            out.append((lo, sz, g + r * sz))
            lo += sz
        return out

    def full_shape(self, kind, local_shape):
        """The parameter's real (un-tensor-parallel) shape."""
        sh = list(local_shape)
        if self.size == 1 or kind == "rep":
            return sh
        if kind == "col":
            sh[1] *= self.size
        else:
            sh[0] *= self.size
        return sh

    def global_shape(self, kind, local_shape):
        R, C = (local_shape[0], int(np.prod(local_shape[1:]))) if len(local_shape) > 1 else (1, local_shape[0])
        if self.size == 1 or kind == "rep":
            return [R, C]
        if kind == "col":
            return [R, C * self.size]
        return [R * self.size, C]

    def rects(self, name, local_shape, start, n):
        """Global rectangles [r0, nr, c0, nc, off] of the local flat range [start, start + n)."""
        kind = param_kind(name) if self.size > 1 else "rep"
        R, C = (local_shape[0], int(np.prod(local_shape[1:]))) if len(local_shape) > 1 else (1, local_shape[0])
        gc0 = self.rank * C if kind == "col" else 0
        blocks = self.blocks(kind, R)

        def grow(j):
            for lo, sz, g in blocks:
                if lo <= j < lo + sz:
                    return g + (j - lo), lo + sz
            raise AssertionError((name, j))

        out, pos, end = [], start, start + n
        while pos < end:
            j, c = divmod(pos, C)
            if c != 0 or end - pos < C:  # partial row
                nc = min(C - c, end - pos)
                g, _ = grow(j)
                out.append([g, 1, gc0 + c, nc, pos - start])
                pos += nc
                continue
            j_end = j + (end - pos) // C
            while j < j_end:
                g, blk_end = grow(j)
                j_stop = min(j_end, blk_end)
                out.append([g, j_stop - j, gc0, C, pos - start])
                pos += (j_stop - j) * C
                j = j_stop
        return out


def _name_map(engine):
    """Parameter name -> checkpoint (global) name: a pipeline stage's decoder layers are
    renumbered from 0 locally (`_dtg_layer_offset` = its first global layer)."""
    off = getattr(engine.module, "_dtg_layer_offset", 0)
    if not off:
        return lambda n: n

    def g(n):
        if n.startswith("layers."):
            i, rest = n[len("layers."):].split(".", 1)
            return f"layers.{int(i) + off}.{rest}"
        return n

    return g


def _replicated_engine(engine) -> bool:
    return getattr(engine, "mode", "fsdp") in ("single", "ddp")


def _writes_shards(engine) -> bool:
    """Whether this rank writes its slices: replicated copies are written once -- by the first
    data-parallel rank of a replicated engine, by replica 0 of a HYBRID_SHARD engine (every
    replica holds the same shards)."""
    if _replicated_engine(engine):
        return getattr(engine, "rank", 0) == 0
    rg = getattr(engine, "replicate_group", None)
    if getattr(engine, "replicas", 1) > 1 and rg is not None and dist.is_initialized():
        return dist.get_rank(rg) == 0
    return True


def snapshot_sharded(engine, global_step=None):
    """Collective: copy this rank's parameter + AdamW-moment slices to host memory and gather
    the slice index of every rank.  Returns (tensors, entry, metadata-or-None) for
    write_sharded; after it returns the device state may change (async checkpointing).

    Replicated copies are written once: with a replicated engine (DDP / single) only the first
    data-parallel rank of each TP group writes, with HYBRID_SHARD only replica 0, and
    TP-replicated parameters (norms) only TP rank 0."""
    rank, world = get_rank(), get_world_size()
    geo = _TPGeom(engine)
    gname = _name_map(engine)
    shapes_local = {n: list(p.shape) for n, p in engine.module.named_parameters()}
    write = _writes_shards(engine)
    skip = getattr(engine.module, "_dtg_ckpt_skip", set())  # e.g. a pipeline's second tied-embedding copy
    pieces = engine.ckpt_pieces()
    tensors, index = {}, []
    for j, (name, start, n, pview, sidx) in enumerate(pieces):
        if not write or name in skip or (geo.size > 1 and geo.rank != 0 and param_kind(name) == "rep"):
            continue
        k = len(index)
        tensors[f"p{k}"] = pview.detach().reshape(-1).to("cpu", copy=True)
        tensors[f"m{k}"] = engine.exp_avg[sidx:sidx + n].to("cpu", copy=True)
        tensors[f"v{k}"] = engine.exp_avg_sq[sidx:sidx + n].to("cpu", copy=True)
        index.append([gname(name), int(n), geo.rects(name, shapes_local[name], int(start), int(n))])
    entry = {"file": _shard_file(rank), "rank": rank, "tp_rank": geo.rank, "index": index}
    if dist.is_initialized() and world > 1:
        gathered = [None] * world
        dist.all_gather_object(gathered, entry)
    else:
        gathered = [entry]
    meta = None
    kind_of = lambda n: param_kind(n) if geo.size > 1 else "rep"
    mine = {gname(n): (geo.global_shape(kind_of(n), sh), geo.full_shape(kind_of(n), sh)) for n, sh in shapes_local.items()}
    if rank == 0:
        files = [f for f in gathered if f["index"]]
        shapes = {}  # from every rank: a pipeline stage knows only its own layers
        if dist.is_initialized() and world > 1:
            allshapes = [None] * world
            dist.gather_object(mine, allshapes, dst=0)
            for d in allshapes:
                shapes.update(d)
        else:
            shapes = mine
        meta = {"format": FORMAT, "world_size": world, "tp_size": geo.size, "step": int(engine.step_count),
                "global_step": global_step, "param_shapes_global": {n: v[0] for n, v in shapes.items()},
                "param_shapes_full": {n: v[1] for n, v in shapes.items()}, "files": files}
    elif dist.is_initialized() and world > 1:
        dist.gather_object(mine, None, dst=0)
    return tensors, entry, meta


def write_sharded(ckpt_dir, tensors, entry, meta):
    """Local file writes only (no collectives): safe on a background thread."""
    ckpt_dir = Path(ckpt_dir)
    ckpt_dir.mkdir(parents=True, exist_ok=True)
    if entry["index"]:
        save_durable(tensors, ckpt_dir / entry["file"])
    if meta is not None:
        with open(ckpt_dir / INDEX, "w") as fp:
            json.dump(meta, fp)
            fp.flush()
            os.fsync(fp.fileno())
    fsync_dir(ckpt_dir)


def save_sharded(ckpt_dir, engine, global_step=None):
    """All ranks: write this rank's parameter + optimizer-state slices; rank 0 writes the index."""
    ckpt_dir = Path(ckpt_dir)
    barrier()
    if get_rank() == 0:
        ckpt_dir.mkdir(parents=True, exist_ok=True)
    barrier()
    write_sharded(ckpt_dir, *snapshot_sharded(engine, global_step))
    barrier()


def read_index(ckpt_dir):
    path = Path(ckpt_dir) / INDEX
    if not path.exists():
        raise FileNotFoundError(f"{ckpt_dir}: no {INDEX} (not a {FORMAT} checkpoint)")
    with open(path) as fp:
        meta = json.load(fp)
    if meta.get("format") != FORMAT:
        raise ValueError(f"{path}: format {meta.get('format')!r}, expected {FORMAT!r}")
    return meta


@torch.no_grad()
def load_sharded(ckpt_dir, engine, load_optimizer: bool = True):
    """Fill this rank's owned parameter (and AdamW-moment) slices from a sharded checkpoint
    written on any data-parallel world size and any tensor-parallel degree.  Raises if a
    parameter is missing, its global shape differs, or any owned element is not covered."""
    ckpt_dir = Path(ckpt_dir)
    meta = read_index(ckpt_dir)
    geo = _TPGeom(engine)
    gname = _name_map(engine)
    shapes_local = {n: list(p.shape) for n, p in engine.module.named_parameters()}
    gshapes = meta["param_shapes_global"]
    for name, sh in shapes_local.items():
        mine = geo.global_shape(param_kind(name) if geo.size > 1 else "rep", sh)
        if gname(name) not in gshapes:
            raise KeyError(f"checkpoint {ckpt_dir} has no parameter {gname(name)!r}")
        if list(gshapes[gname(name)]) != mine:
            raise ValueError(f"{gname(name)}: checkpoint global shape {gshapes[gname(name)]} != model's {mine}")
    stored = {}  # name -> [(file, key, rect)]
    seen = set()  # identical rectangles stored twice (replicas of a pre-fix HYBRID save): read once
    for f in meta["files"]:
        for k, (name, n, rects) in enumerate(f["index"]):
            for rc in rects:
                key = (name, tuple(rc[:4]))
                if key in seen:
                    continue
                seen.add(key)
                stored.setdefault(name, []).append((f["file"], k, rc))
    cache = {}

    def get(fname):
        if fname not in cache:
            if not (ckpt_dir / fname).exists():
                raise FileNotFoundError(f"checkpoint shard {ckpt_dir / fname} is missing")
            cache[fname] = torch.load(ckpt_dir / fname, weights_only=True, mmap=True)
        return cache[fname]

    for name, start, n, pview, sidx in engine.ckpt_pieces():
        dsts = [pview.reshape(-1)]
        if load_optimizer:
            dsts += [engine.exp_avg[sidx:sidx + n], engine.exp_avg_sq[sidx:sidx + n]]
        covered = 0
        for tr0, tnr, tc0, tnc, toff in geo.rects(name, shapes_local[name], int(start), int(n)):
            for fname, k, (sr0, snr, sc0, snc, soff) in stored.get(gname(name), []):
                r_lo, r_hi = max(tr0, sr0), min(tr0 + tnr, sr0 + snr)
                c_lo, c_hi = max(tc0, sc0), min(tc0 + tnc, sc0 + snc)
                if r_lo >= r_hi or c_lo >= c_hi:
                    continue
                t = get(fname)
                for dst, key in zip(dsts, ("p", "m", "v")):
                    src = t[f"{key}{k}"][soff:soff + snr * snc].view(snr, snc)[r_lo - sr0:r_hi - sr0, c_lo - sc0:c_hi - sc0]
                    dst[toff:toff + tnr * tnc].view(tnr, tnc)[r_lo - tr0:r_hi - tr0, c_lo - tc0:c_hi - tc0].copy_(src)
                covered += (r_hi - r_lo) * (c_hi - c_lo)
        if covered != n:
            raise RuntimeError(f"checkpoint {ckpt_dir} covers {covered} of the {n} elements this rank owns "
                               f"of {name!r} (elements [{start}, {start + n}))")
    if load_optimizer:
        engine.step_count = int(meta["step"])
    # replicated engines must see identical parameters everywhere (ZeRO all-gathers its slices)
    sync = getattr(engine, "sync_params_after_load", None)
    if sync is not None:
        sync()
    barrier()
    return meta


# ------------------------------------------------------------------------------ export / import
def _stored_rects(meta):
    stored, seen = {}, set()
    for f in meta["files"]:
        for k, (name, n, rects) in enumerate(f["index"]):
            for rc in rects:
                key = (name, tuple(rc[:4]))
                if key not in seen:
                    seen.add(key)
                    stored.setdefault(name, []).append((f["file"], k, rc))
    return stored


def iter_full_params(ckpt_dir, what=("p",)):
    """Yield (name, {"p": param[, "m": exp_avg, "v": exp_avg_sq]}) of a dtg-sharded-v2
    checkpoint, one parameter at a time in its real (un-sharded, un-tensor-parallel) shape,
    assembled on the host from the memory-mapped shard files -- peak memory is one parameter,
    not the model.  Raises if any element of a parameter is not stored."""
    ckpt_dir = Path(ckpt_dir)
    meta = read_index(ckpt_dir)
    stored = _stored_rects(meta)
    files = {}

    def get(fname):
        if fname not in files:
            files[fname] = torch.load(ckpt_dir / fname, weights_only=True, mmap=True)
        return files[fname]

    full_shapes = meta.get("param_shapes_full", {})
    for name, (R, C) in meta["param_shapes_global"].items():
        outs, covered = {}, 0
        for fname, k, (r0, nr, c0, nc, off) in stored.get(name, []):
            t = get(fname)
            for key in what:
                src = t[f"{key}{k}"]
                if key not in outs:
                    outs[key] = torch.empty((R, C), dtype=src.dtype)
                outs[key][r0:r0 + nr, c0:c0 + nc].copy_(src[off:off + nr * nc].view(nr, nc))
            covered += nr * nc
        if covered != R * C:
            raise RuntimeError(f"{ckpt_dir}: parameter {name!r} is only {covered} of {R * C} elements covered")
        shape = full_shapes.get(name) or ([C] if R == 1 else [R, C])  # pre-`param_shapes_full` indexes
        yield name, {key: v.view(*shape) for key, v in outs.items()}


def consolidate_sharded(ckpt_dir, with_optimizer: bool = False):
    """Full host state dict {name: param} (and, with_optimizer, {name: (exp_avg, exp_avg_sq)})."""
    what = ("p", "m", "v") if with_optimizer else ("p",)
    params, moments = {}, {}
    for name, d in iter_full_params(ckpt_dir, what):
        params[name] = d["p"]
        if with_optimizer:
            moments[name] = (d["m"], d["v"])
    return (params, moments) if with_optimizer else params


def write_single_shard(ckpt_dir, params: dict, moments: dict = None, step: int = 0, global_step=None):
    """Write full parameters (real shapes, this framework's names) as a one-shard
    dtg-sharded-v2 checkpoint: world 1, no TP.  `load_sharded` reshards it onto any
    (data-parallel x tensor-parallel) layout, so this is the import path for weights trained
    elsewhere (HF safetensors -> hf_compat -> here).  Missing moments are written as zeros."""
    ckpt_dir = Path(ckpt_dir)
    ckpt_dir.mkdir(parents=True, exist_ok=True)
    tensors, index, gsh, fsh = {}, [], {}, {}
    for k, (name, p) in enumerate(params.items()):
        p = p.detach().contiguous()
        R, C = (p.shape[0], int(np.prod(p.shape[1:]))) if p.dim() > 1 else (1, p.shape[0])
        m, v = (moments or {}).get(name, (None, None))
        tensors[f"p{k}"] = p.reshape(-1).cpu()
        tensors[f"m{k}"] = (m.reshape(-1).to(p.dtype) if m is not None else torch.zeros(p.numel(), dtype=p.dtype)).cpu()
        tensors[f"v{k}"] = (v.reshape(-1).to(p.dtype) if v is not None else torch.zeros(p.numel(), dtype=p.dtype)).cpu()
        index.append([name, int(p.numel()), [[0, R, 0, C, 0]]])
        gsh[name], fsh[name] = [R, C], list(p.shape)
    torch.save(tensors, ckpt_dir / _shard_file(0))
    meta = {"format": FORMAT, "world_size": 1, "tp_size": 1, "step": int(step), "global_step": global_step,
            "param_shapes_global": gsh, "param_shapes_full": fsh,
            "files": [{"file": _shard_file(0), "rank": 0, "tp_rank": 0, "index": index}]}
    with open(ckpt_dir / INDEX, "w") as fp:
        json.dump(meta, fp)
    return meta


# ------------------------------------------------------------------------------ high level
def _any_failed(err) -> bool:
    """Collective: did the checkpoint write fail on ANY rank?  Every rank then raises together,
    instead of the healthy ranks waiting at the next barrier for a rank that already left."""
    if not (dist.is_initialized() and get_world_size() > 1) or dist.get_backend() == "fake":
        return err is not None
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    t = torch.tensor([int(err is not None)], dtype=torch.int32, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return bool(t.item())


class CheckpointManager:
    """Save/resume in the reference's layout. `style` in {"full", "dp", "sharded"}.

    Every save goes through the `.pending/` journal (see `commit_pending`): the previous
    checkpoint stays valid until the new one is complete.  `async_save=True`:
    `save()` only snapshots the state to host memory (device -> host copies plus the small
    metadata collectives) and returns; a background thread writes the files into .pending.  The
    next `save()` or `finalize()` joins the writer on every rank, meets at a barrier, and rank 0
    commits."""

    PENDING = PENDING

    def __init__(self, exp_dir, engine, optimizer, lr_scheduler, style: str, local_rank: int = 0,
                 async_save: bool = False, fmt: str = "dcp"):
        """fmt: the `checkpoint/` format of the "dp" / "sharded" styles -- "dcp" (torch DCP, the
        reference's tree; train/dcp_ckpt.py) or "dtg" (dtg-sharded-v2).  Loading reads either.
        An async DCP save snapshots the chunks into reused pinned host buffers and runs DCP's
        planning collectives and file writes on the writer thread over a dedicated gloo group
        (created here, collectively), so the training thread's process group is never shared."""
        assert fmt in ("dcp", "dtg"), fmt
        self.exp_dir = Path(exp_dir)
        self.engine, self.optimizer, self.lr_scheduler = engine, optimizer, lr_scheduler
        self.style = style
        self.local_rank = local_rank
        self.fmt = fmt
        self.async_save = async_save
        self._writer = None   # background thread of the pending save
        self._host_pool = None  # dcp_ckpt.HostPool of the async DCP snapshots (reused)
        self._ckpt_pg = None    # gloo group of the async DCP writer thread
        if (async_save and fmt == "dcp" and style != "full" and dist.is_initialized() and get_world_size() > 1
                and dist.get_backend() != "fake"):  # a DTG_FAKE_WORLD rehearsal never saves
            self._ckpt_pg = dist.new_group(backend="gloo")
        self._pending = None  # (state, lr_scheduler state, rng state) to publish on finalize
        self._error = None

    def _snapshot_host(self, global_step=None):
        """Collective part of a save: everything the writer needs, on the host."""
        jobs = []  # (relative path, object) for torch.save; sharded handled separately
        shard = None
        if self.style == "full":
            if get_rank() == 0:
                jobs.append(("model.pt", self.engine.full_state_dict()))
                jobs.append(("optimizer.pt", _to_cpu(self.optimizer.state_dict())))
        else:
            if self.style == "dp":
                sd = self.engine.full_state_dict()
                if get_rank() == 0:
                    jobs.append(("model.pt", sd))
            if self.fmt == "dcp" and self.async_save:
                from .dcp_ckpt import HostPool, snapshot_dcp

                if self._host_pool is None:
                    self._host_pool = HostPool()
                shard = ("dcp-snap", snapshot_dcp(self.engine, self.optimizer, self.engine.module.config, global_step,
                                                  host_pool=self._host_pool))
            elif self.fmt == "dcp":
                shard = ("dcp", global_step)
            else:
                shard = snapshot_sharded(self.engine, global_step)
        return jobs, shard

    def _write_pending(self, jobs, shard):
        try:
            pend = self.exp_dir / self.PENDING
            pend.mkdir(parents=True, exist_ok=True)
            for rel, obj in jobs:
                save_durable(obj, pend / rel)
            if shard is not None and shard[0] == "dcp":
                from .dcp_ckpt import save_dcp

                save_dcp(pend / "checkpoint", self.engine, self.optimizer, self.engine.module.config, shard[1])
            elif shard is not None and shard[0] == "dcp-snap":
                from .dcp_ckpt import write_dcp

                write_dcp(pend / "checkpoint", shard[1], process_group=self._ckpt_pg)
            elif shard is not None:
                write_sharded(pend / "checkpoint", *shard)
        except BaseException as e:  # surfaced by finalize() on the main thread
            self._error = e

    def _publish(self, state, sched_sd, rng):
        """Rank 0: the small files into .pending, then the atomic commit."""
        pend = self.exp_dir / self.PENDING
        pend.mkdir(parents=True, exist_ok=True)
        save_durable(sched_sd, pend / "lr_scheduler.pt")
        save_durable(rng.obj if isinstance(rng, _RngBox) else rng, pend / "rng.pt")
        with open(pend / "state.json", "w") as fp:
            json.dump(state, fp)
            fp.flush()
            os.fsync(fp.fileno())
        commit_pending(self.exp_dir)

    def finalize(self):
        """Publish the pending async save (collective: call on every rank)."""
        if self._writer is None:
            return
        self._writer.join()
        self._writer = None
        err, self._error = self._error, None
        if _any_failed(err):
            self._pending = None  # the half-written .pending is discarded by the next save / start
            raise RuntimeError("async checkpoint write failed" + ("" if err else " on another rank")) from err
        barrier()
        if get_rank() == 0:
            self._publish(*self._pending)
        self._pending = None
        barrier()

    def _begin(self):
        """Collective: a clean .pending (a stale one from a crashed save is discarded)."""
        import shutil

        barrier()
        if get_rank() == 0:
            shutil.rmtree(self.exp_dir / self.PENDING, ignore_errors=True)
            (self.exp_dir / self.PENDING).mkdir(parents=True, exist_ok=True)
        barrier()

    def save(self, state: dict):
        if self.async_save:
            import threading

            self.finalize()
            self._begin()
            jobs, shard = self._snapshot_host(state.get("global_step"))
            if get_rank() == 0:
                box = _RngBox()
                save_rng(box)
                self._pending = (dict(state), _to_cpu(self.lr_scheduler.state_dict()), box.obj)
            else:
                self._pending = (None, None, None)
            self._writer = threading.Thread(target=self._write_pending, args=(jobs, shard), daemon=False)
            self._writer.start()
            return
        self._begin()
        jobs, shard = self._snapshot_host(state.get("global_step"))
        self._write_pending(jobs, shard)
        err, self._error = self._error, None
        if _any_failed(err):
            raise RuntimeError("checkpoint write failed" + ("" if err else " on another rank")) from err
        barrier()
        if get_rank() == 0:
            box = _RngBox()
            save_rng(box)
            self._publish(dict(state), self.lr_scheduler.state_dict(), box.obj)
        barrier()

    def load(self) -> dict:
        d = self.exp_dir
        dev = self.engine.space.param_buf.device if hasattr(self.engine, "space") else self.engine.device
        if self.style == "full":
            sd = torch.load(d / "model.pt", map_location=dev, weights_only=True)
            self.engine.module.load_state_dict(sd)
            self.optimizer.load_state_dict(torch.load(d / "optimizer.pt", map_location=dev, weights_only=True))
            meta = None
        else:
            from .dcp_ckpt import is_dcp_dir, load_dcp

            if is_dcp_dir(d / "checkpoint"):
                meta = load_dcp(d / "checkpoint", self.engine, self.engine.module.config)
            else:
                meta = load_sharded(d / "checkpoint", self.engine)
        self.lr_scheduler.load_state_dict(torch.load(d / "lr_scheduler.pt", weights_only=True))
        # The sharded / per-rank layouts restore the AdamW moments but not the optimizer's
        # param_groups, and chainable schedulers (CosineAnnealingLR) compute the next lr FROM the
        # group's current lr: without this the resumed run restarted the recursion from the
        # initial lr (a TP=2 -> TP=1 resume on the GPU logged step 4 at step 3's lr, and the whole
        # tail of the schedule scaled by lr0 / lr(resume step)).
        for g, lr in zip(self.optimizer.param_groups, self.lr_scheduler.get_last_lr()):
            g["lr"] = lr
        if (d / "rng.pt").exists():
            load_rng(d / "rng.pt", self.local_rank)
        with open(d / "state.json") as fp:
            state = json.load(fp)
        if meta is not None and meta.get("global_step") is not None and meta["global_step"] != state.get("global_step"):
            raise RuntimeError(f"{d}: checkpoint/ holds step {meta['global_step']} but state.json says "
                               f"{state.get('global_step')} (interrupted save?)")
        barrier()
        return state
