"""Checkpoint / resume.

Directory layout under `{save_dir}/{experiment_name}/` follows the reference per chapter:
  * full (01, rime):  model.pt, optimizer.pt, lr_scheduler.pt, state.json, rng.pt
  * dp   (02):        model.pt (rank 0), lr_scheduler.pt, state.json, rng.pt + the optimizer
                      state as a sharded `checkpoint/` (the reference never saved it and then
                      crashed on resume)
  * sharded (04-07):  checkpoint/ (.metadata + one file per rank), lr_scheduler.pt, state.json, rng.pt

Sharded format (a DCP-like layout, resharding-capable): every rank writes
`checkpoint/__{rank}_0.distcp` holding, for each parameter slice it owns, the parameter values
and both AdamW moments (plain tensors: loadable with `torch.load(weights_only=True)`), and rank 0
writes `checkpoint/.metadata` (JSON) with every file's slice index.  On load each rank copies
the overlap of every stored slice with the slices it owns now, so a checkpoint written by W
ranks loads on W' ranks (FSDP, ZeRO and DDP layouts alike); TP shards are matched by tp rank.
Barriers bracket every save (reference C2) so no rank reads a half-written directory.
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
def _tp_rank(engine):
    tp = getattr(engine.module, "tp", None)
    return (tp.rank, tp.size) if tp is not None and tp.enabled else (0, 1)


def snapshot_sharded(engine):
    """Collective: copy this rank's parameter + AdamW-moment slices to host memory and gather
    the slice index of every rank.  Returns (tensors, entry, metadata-or-None) for
    write_sharded; after it returns the device state may change (async checkpointing)."""
    rank, world = get_rank(), get_world_size()
    pieces = engine.ckpt_pieces()
    tensors, index = {}, []
    for j, (name, start, n, pview, sidx) in enumerate(pieces):
        tensors[f"p{j}"] = pview.detach().reshape(-1).to("cpu", copy=True)
        tensors[f"m{j}"] = engine.exp_avg[sidx:sidx + n].to("cpu", copy=True)
        tensors[f"v{j}"] = engine.exp_avg_sq[sidx:sidx + n].to("cpu", copy=True)
        index.append([name, int(start), int(n)])
    tp_rank, tp_size = _tp_rank(engine)
    fname = f"__{rank}_0.distcp"
    entry = {"file": fname, "rank": rank, "tp_rank": tp_rank, "index": index}
    if dist.is_initialized() and world > 1:
        gathered = [None] * world
        dist.all_gather_object(gathered, entry)
    else:
        gathered = [entry]
    meta = None
    if rank == 0:
        shapes = {n: list(p.shape) for n, p in engine.module.named_parameters()}
        meta = {"world_size": world, "tp_size": tp_size, "step": int(engine.step_count), "files": gathered,
                "param_shapes_tp_local": shapes, "format": "dtg-sharded-v1"}
    return tensors, entry, meta


def write_sharded(ckpt_dir, tensors, entry, meta):
    """Local file writes only (no collectives): safe on a background thread."""
    ckpt_dir = Path(ckpt_dir)
    ckpt_dir.mkdir(parents=True, exist_ok=True)
    torch.save(tensors, ckpt_dir / entry["file"])
    if meta is not None:
        with open(ckpt_dir / ".metadata", "w") as fp:
            json.dump(meta, fp)


def save_sharded(ckpt_dir, engine):
    """All ranks: write this rank's parameter + optimizer-state slices; rank 0 writes metadata."""
    ckpt_dir = Path(ckpt_dir)
    barrier()
    if get_rank() == 0:
        ckpt_dir.mkdir(parents=True, exist_ok=True)
    barrier()
    write_sharded(ckpt_dir, *snapshot_sharded(engine))
    barrier()


@torch.no_grad()
def load_sharded(ckpt_dir, engine, load_optimizer: bool = True):
    ckpt_dir = Path(ckpt_dir)
    with open(ckpt_dir / ".metadata") as fp:
        meta = json.load(fp)
    tp_rank, tp_size = _tp_rank(engine)
    assert meta.get("tp_size", 1) == tp_size, "checkpoint tensor-parallel degree differs from the run's"
    # stored slices by parameter name: (file, key index, start, n)
    stored = {}
    for f in meta["files"]:
        if f.get("tp_rank", 0) != tp_rank:
            continue
        for j, (name, start, n) in enumerate(f["index"]):
            stored.setdefault(name, []).append((f["file"], j, start, n))
    cache = {}

    def get(fname):
        if fname not in cache:
            cache[fname] = torch.load(ckpt_dir / fname, weights_only=True, mmap=True)
        return cache[fname]

    for name, start, n, pview, sidx in engine.ckpt_pieces():
        flat = pview.reshape(-1)
        for fname, j, s2, n2 in stored.get(name, []):
            lo, hi = max(start, s2), min(start + n, s2 + n2)
            if lo >= hi:
                continue
            t = get(fname)
            flat[lo - start:hi - start].copy_(t[f"p{j}"][lo - s2:hi - s2])
            if load_optimizer:
                engine.exp_avg[sidx + lo - start:sidx + hi - start].copy_(t[f"m{j}"][lo - s2:hi - s2])
                engine.exp_avg_sq[sidx + lo - start:sidx + hi - start].copy_(t[f"v{j}"][lo - s2:hi - s2])
    if load_optimizer:
        engine.step_count = int(meta["step"])
    # replicated engines must see identical parameters everywhere (ZeRO all-gathers its slices)
    sync = getattr(engine, "sync_params_after_load", None)
    if sync is not None:
        sync()
    barrier()


# ------------------------------------------------------------------------------ high level
class CheckpointManager:
    """Save/resume in the reference's layout. `style` in {"full", "dp", "sharded"}.

    `async_save=True`: `save()` only snapshots the state to host memory (device
    -> host copies plus the small metadata collectives) and returns; a background thread
    writes the files into `{exp_dir}/.pending/`.  The next `save()` or `finalize()` joins the
    writer on every rank, meets at a barrier, and rank 0 moves the finished files into place and
    writes `state.json` LAST -- resume keys on state.json, so an interrupted write is never
    mistaken for a checkpoint."""

    PENDING = ".pending"

    def __init__(self, exp_dir, engine, optimizer, lr_scheduler, style: str, local_rank: int = 0,
                 async_save: bool = False):
        self.exp_dir = Path(exp_dir)
        self.engine, self.optimizer, self.lr_scheduler = engine, optimizer, lr_scheduler
        self.style = style
        self.local_rank = local_rank
        self.async_save = async_save
        self._writer = None   # background thread of the pending save
        self._pending = None  # (state, lr_scheduler state, rng state) to publish on finalize
        self._error = None

    # ------------------------------------------------------------------ async path
    def _snapshot_host(self):
        """Collective part of a save: everything the writer thread needs, on the host."""
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
            shard = snapshot_sharded(self.engine)
        return jobs, shard

    def _write_pending(self, jobs, shard):
        try:
            pend = self.exp_dir / self.PENDING
            pend.mkdir(parents=True, exist_ok=True)
            for rel, obj in jobs:
                torch.save(obj, pend / rel)
            if shard is not None:
                write_sharded(pend / "checkpoint", *shard)
        except BaseException as e:  # surfaced by finalize() on the main thread
            self._error = e

    def finalize(self):
        """Publish the pending async save (collective: call on every rank)."""
        if self._writer is None:
            return
        self._writer.join()
        self._writer = None
        err, self._error = self._error, None
        if err is not None:
            raise RuntimeError("async checkpoint write failed") from err
        barrier()
        if get_rank() == 0:
            import shutil

            pend, d = self.exp_dir / self.PENDING, self.exp_dir
            state, sched_sd, rng = self._pending
            for item in pend.iterdir():
                dst = d / item.name
                if dst.is_dir():
                    shutil.rmtree(dst)
                os.replace(item, dst)
            torch.save(sched_sd, d / "lr_scheduler.pt")
            torch.save(rng, d / "rng.pt")
            with open(d / "state.json", "w") as fp:
                json.dump(state, fp)
            shutil.rmtree(pend, ignore_errors=True)
        self._pending = None
        barrier()

    def save(self, state: dict):
        if self.async_save:
            import threading

            self.finalize()
            barrier()
            jobs, shard = self._snapshot_host()
            if get_rank() == 0:
                box = _RngBox()
                save_rng(box)
                self._pending = (dict(state), _to_cpu(self.lr_scheduler.state_dict()), box.obj)
            else:
                self._pending = (None, None, None)
            self._writer = threading.Thread(target=self._write_pending, args=(jobs, shard), daemon=False)
            self._writer.start()
            return
        rank = get_rank()
        d = self.exp_dir
        barrier()
        if self.style == "full":
            if rank == 0:
                torch.save(self.engine.full_state_dict(), d / "model.pt")
                torch.save(self.optimizer.state_dict(), d / "optimizer.pt")
        elif self.style == "dp":
            sd = self.engine.full_state_dict()
            if rank == 0:
                torch.save(sd, d / "model.pt")
            save_sharded(d / "checkpoint", self.engine)
        else:
            save_sharded(d / "checkpoint", self.engine)
        if rank == 0:
            torch.save(self.lr_scheduler.state_dict(), d / "lr_scheduler.pt")
            save_rng(d / "rng.pt")
            with open(d / "state.json", "w") as fp:
                json.dump(state, fp)
        barrier()

    def load(self) -> dict:
        d = self.exp_dir
        dev = self.engine.space.param_buf.device if hasattr(self.engine, "space") else self.engine.device
        if self.style == "full":
            sd = torch.load(d / "model.pt", map_location=dev, weights_only=True)
            self.engine.module.load_state_dict(sd)
            self.optimizer.load_state_dict(torch.load(d / "optimizer.pt", map_location=dev, weights_only=True))
        else:
            load_sharded(d / "checkpoint", self.engine)
        self.lr_scheduler.load_state_dict(torch.load(d / "lr_scheduler.pt", weights_only=True))
        if (d / "rng.pt").exists():
            load_rng(d / "rng.pt", self.local_rank)
        with open(d / "state.json") as fp:
            state = json.load(fp)
        barrier()
        return state
