"""torch.distributed.checkpoint (DCP) as the sharded chapters' native on-disk format
(`--ckpt-format dcp`, the default for chapters 02 and 04-07).

The reference saves `{exp_dir}/checkpoint` from every rank with
`dcp.save({"model": model_sd, "optimizer": optim_sd}, checkpoint_id=exp_dir / "checkpoint")`
(/root/reference/04-fully-sharded-data-parallel/train_llm.py:121-154, 249-263;
06-tensor-parallel/train_llm.py:177-190, 283-295): a `.metadata` file plus one `__<rank>_0.distcp`
file per rank, with HF parameter names (`model.layers.0.self_attn.q_proj.weight`, ...) and torch
AdamW's state layout (`optimizer.state.<fqn>.{exp_avg, exp_avg_sq, step}`, `param_groups`).
This module writes exactly that tree from this framework's engines, without DTensors or
ShardedTensors:

* every rank describes the slices it owns (FSDP flat-shard ranges, ZeRO bucket slices,
  tensor-parallel row / column blocks -- `checkpoint._TPGeom.rects`, rectangles in GLOBAL
  parameter coordinates) as DCP chunks: offsets + sizes in the HF tensor's real shape.  The
  fused `qkv_proj` / `gate_up_proj` rows split into their q / k / v and gate / up tensors at the
  row boundaries, so a chunk never straddles two HF tensors;
* a custom `SavePlanner` hands those chunks to DCP's FileSystemWriter (one file per rank,
  fsynced), and rank 0 adds the `param_groups` with the full AdamW hyper-parameters;
* resume is `dcp.load` with a custom `LoadPlanner` whose destination chunks are views into the
  engine's own parameter / moment buffers: DCP's resharding reads the overlap of every stored
  chunk, so a checkpoint written on W x TP a loads on W' x TP b (data-parallel world, tensor-
  parallel degree, pipeline stages, FSDP / ZeRO / DDP layouts alike).  A destination element no
  stored chunk covers fails the load.

`torch.distributed.checkpoint.format_utils.dcp_to_torch_save(exp_dir / "checkpoint", "full.pt")`
reads a training run's checkpoint directly (the reference's README recipe).  The small
`checkpoint/dtg.json` records the step counters (DCP ignores files it did not write).
The previous format (`dtg-sharded-v2`: index.json + shard_rNNNNN.pt) stays readable.
"""
from __future__ import annotations

import io
import json
import os
from pathlib import Path

import torch
import torch.distributed as dist

FORMAT = "dcp"
META = "dtg.json"


def is_dcp_dir(ckpt_dir) -> bool:
    return (Path(ckpt_dir) / ".metadata").exists()


# ------------------------------------------------------------------------------ naming
class _Names:
    """This framework's parameter (global name, global [R, C] rectangle) -> HF-named DCP chunks."""

    def __init__(self, cfg):
        from ..models.config import LlamaConfig

        self.cfg = cfg
        self.llama = isinstance(cfg, LlamaConfig)

    def split(self, name, full_shape, rect):
        """[(hf_fqn, hf_shape, offsets, sizes, (r_lo, r_hi))] for rectangle rect = [r0, nr, c0, nc,
        off] (global rows x flattened columns) of parameter `name`; (r_lo, r_hi) are the rect's
        rows that chunk covers."""
        r0, nr, c0, nc, _ = rect
        shape = list(full_shape)
        if not self.llama:
            return [(name, shape, *_chunk(shape, r0, nr, c0, nc), (r0, r0 + nr))]
        cfg = self.cfg
        parts = None  # [(HF name, first global row, rows)]
        if name.endswith("self_attn.qkv_proj.weight") or name.endswith("self_attn.qkv_proj.bias"):
            d, nq, nkv = cfg.head_dim, cfg.num_attention_heads, cfg.num_key_value_heads
            pre, leaf = name.rsplit("qkv_proj.", 1)
            parts = [(f"{pre}q_proj.{leaf}", 0, nq * d), (f"{pre}k_proj.{leaf}", nq * d, nkv * d),
                     (f"{pre}v_proj.{leaf}", (nq + nkv) * d, nkv * d)]
        elif name.endswith("mlp.gate_up_proj.weight"):
            i = shape[0] // 2
            pre = name[: -len("gate_up_proj.weight")]
            parts = [(f"{pre}gate_proj.weight", 0, i), (f"{pre}up_proj.weight", i, i)]
        if parts is None:
            hf = name if name == "lm_head.weight" else "model." + name
            return [(hf, shape, *_chunk(shape, r0, nr, c0, nc), (r0, r0 + nr))]
        out = []
        for hf, g0, rows in parts:
            lo, hi = max(r0, g0), min(r0 + nr, g0 + rows)
            if lo >= hi:
                continue
            # this framework's q/k/v bias is [N, 1]; HF's is [N]
            sub = [rows] if name.endswith("bias") else [rows] + shape[1:]
            out.append(("model." + hf, sub, *_chunk(sub, lo - g0, hi - lo, c0, nc, rows_1d=len(sub) == 1), (lo, hi)))
        return out


def _chunk(shape, r0, nr, c0, nc, rows_1d=False):
    """(offsets, sizes) of a global [rows x flattened cols] rectangle in a tensor of `shape`.  A 1-D
    parameter (norm weight) is one global row [1, C]; `rows_1d`: a 1-D HF tensor stored here as
    N rows of one column (the [N, 1] q/k/v biases)."""
    if len(shape) == 2:
        return [r0, c0], [nr, nc]
    if len(shape) == 1:
        return ([r0], [nr]) if rows_1d else ([c0], [nc])
    raise ValueError(f"DCP chunks: {len(shape)}-D parameters are not supported")


def _chunks(engine, cfg, keep=None):
    """This rank's DCP chunks: [(hf_fqn, hf_shape, offsets, sizes, {"p" | "m" | "v": view})] of the
    owned pieces whose local parameter name passes `keep`.  Views index the engine's live buffers
    (reads for a save, in-place writes for a load)."""
    from .checkpoint import _TPGeom, _name_map, param_kind

    geo = _TPGeom(engine)
    gname = _name_map(engine)
    shapes_local = {n: list(p.shape) for n, p in engine.module.named_parameters()}
    names = _Names(cfg)
    out = []
    kind_of = (lambda n: param_kind(n)) if geo.size > 1 else (lambda n: "rep")
    for name, start, n, pview, sidx in engine.ckpt_pieces():
        if keep is not None and not keep(name):
            continue
        full = geo.full_shape(kind_of(name), shapes_local[name])
        flat = {"p": pview.detach().reshape(-1), "m": engine.exp_avg[sidx:sidx + n],
                "v": engine.exp_avg_sq[sidx:sidx + n]}
        for rect in geo.rects(name, shapes_local[name], int(start), int(n)):
            r0, nr, c0, nc, off = rect
            for hf, hshape, offs, sizes, (lo, hi) in names.split(gname(name), full, rect):
                views = {k: t[off:off + nr * nc].view(nr, nc)[lo - r0:hi - r0] for k, t in flat.items()}
                views = {k: v.reshape(sizes) for k, v in views.items()}
                out.append((hf, hshape, list(offs), list(sizes), views))
    return out


# ------------------------------------------------------------------------------ save
def _planners():
    from torch.distributed.checkpoint.default_planner import DefaultLoadPlanner, DefaultSavePlanner
    from torch.distributed.checkpoint.metadata import ChunkStorageMetadata, MetadataIndex, TensorProperties
    from torch.distributed.checkpoint.planner import (SavePlan, TensorWriteData, WriteItem, WriteItemType,
                                                      LoadPlan)
    from torch.distributed.checkpoint.planner_helpers import create_read_items_for_chunk_list

    class ChunkSavePlanner(DefaultSavePlanner):
        """Writes precomputed chunks (tensors) and objects (coordinator) under flat DCP keys."""

        def __init__(self, tensors, objects, mappings):
            super().__init__()
            self._tensors = tensors    # [(flat key, global shape, offsets, tensor)]
            self._objects = objects    # {flat key: picklable object}
            self._mappings = mappings  # {flat key: nested path}
            self._lookup = {}

        def set_up_planner(self, state_dict, storage_meta=None, is_coordinator=False):
            self.state_dict = {}
            self.is_coordinator = is_coordinator

        def create_local_plan(self):
            items = []
            for key, gshape, offs, t in self._tensors:
                props = TensorProperties.create_from_tensor(t)
                chunk = ChunkStorageMetadata(offsets=torch.Size(offs), sizes=t.size())
                wtype = WriteItemType.SHARD if len(gshape) else WriteItemType.TENSOR
                items.append(WriteItem(index=MetadataIndex(key, torch.Size(offs)), type=wtype,
                                       tensor_data=TensorWriteData(chunk=chunk, properties=props,
                                                                   size=torch.Size(gshape))))
                self._lookup[(key, tuple(offs))] = t
            for key in self._objects:
                items.append(WriteItem(index=MetadataIndex(key), type=WriteItemType.BYTE_IO))
            self.plan = SavePlan(items, planner_data=dict(self._mappings))
            return self.plan

        def resolve_data(self, write_item):
            key = write_item.index.fqn
            if write_item.type == WriteItemType.BYTE_IO:
                buf = io.BytesIO()
                torch.save(self._objects[key], buf)
                return buf
            t = self._lookup[(key, tuple(write_item.index.offset or ()))]
            return t.detach().to("cpu").contiguous()

    class ChunkLoadPlanner(DefaultLoadPlanner):
        """Reads stored chunks into destination views (any stored layout -> this rank's layout)."""

        def __init__(self, dests, scalars):
            super().__init__()
            self._dests = dests      # [(flat key, global shape, offsets, view)]
            self._scalars = scalars  # {flat key: 0-d tensor} filled from the checkpoint
            self._lookup = {}
            self.covered = {}

        def set_up_planner(self, state_dict, metadata=None, is_coordinator=False):
            self.state_dict = {}
            self.metadata = metadata
            self.is_coordinator = is_coordinator

        def create_local_plan(self):
            md = self.metadata.state_dict_metadata
            items = []
            for key, gshape, offs, view in self._dests:
                if key not in md:
                    raise KeyError(f"DCP checkpoint has no tensor {key!r}")
                if list(md[key].size) != list(gshape):
                    raise ValueError(f"{key}: checkpoint shape {list(md[key].size)} != model's {list(gshape)}")
                chunk = ChunkStorageMetadata(offsets=torch.Size(offs), sizes=view.size())
                got = create_read_items_for_chunk_list(key, md[key], [chunk])
                self._lookup[(key, tuple(offs))] = view
                vol = 0
                for it in got:
                    n = 1
                    for x in it.lengths:
                        n *= int(x)
                    vol += n
                if vol != view.numel():
                    raise RuntimeError(f"DCP checkpoint covers {vol} of the {view.numel()} elements of {key} "
                                       f"this rank owns at offsets {offs}")
                items += got
            for key, t in self._scalars.items():
                if key not in md:
                    raise KeyError(f"DCP checkpoint has no tensor {key!r}")
                chunk = ChunkStorageMetadata(offsets=torch.Size([]), sizes=torch.Size([]))
                items += create_read_items_for_chunk_list(key, md[key], [chunk])
                self._lookup[(key, ())] = t
            self.plan = LoadPlan(items)
            return self.plan

        def create_global_plan(self, global_plan):
            return global_plan

        def resolve_tensor(self, read_item):
            from torch.distributed._shard._utils import narrow_tensor_by_index

            dst = self._lookup[(read_item.dest_index.fqn, tuple(read_item.dest_index.offset or ()))]
            return narrow_tensor_by_index(dst, read_item.dest_offsets, read_item.lengths)

        def commit_tensor(self, read_item, tensor):
            pass  # the reader copied into a view of the destination

    return ChunkSavePlanner, ChunkLoadPlanner


def _adamw_group(optimizer):
    """torch AdamW's full param_group (without "params"): the hyper-parameters of this run, plus
    every extra plain-valued key the optimizer carries (e.g. the scheduler's `initial_lr`, which
    the reference's `get_state_dict` also asks for on resume)."""
    g = optimizer.param_groups[0] if optimizer is not None else {}
    out = {"lr": float(g.get("lr", 0.0)), "betas": tuple(g.get("betas", (0.9, 0.999))), "eps": float(g.get("eps", 1e-8)),
           "weight_decay": float(g.get("weight_decay", 0.01)), "amsgrad": False, "foreach": None, "maximize": False,
           "capturable": False, "differentiable": False, "fused": True, "decoupled_weight_decay": True}
    for k, v in g.items():
        if k not in out and k != "params" and isinstance(v, (bool, int, float, str, tuple, type(None))):
            out[k] = v
    return out


class DcpSnapshot:
    """Everything one rank writes for a DCP save: [(flat key, global shape, offsets, tensor)] chunks,
    rank 0's param_group objects, the key -> nested-path mappings and the dtg.json record."""

    def __init__(self, tensors, objects, mappings, meta, multi):
        self.tensors, self.objects, self.mappings, self.meta, self.multi = tensors, objects, mappings, meta, multi


def snapshot_dcp(engine, optimizer, cfg, global_step=None, host_pool=None) -> DcpSnapshot:
    """Collective (every rank): describe this rank's part of a DCP save of {"model": ...,
    "optimizer": ...} in the reference's layout.  With `host_pool` (a HostPool) every chunk is
    COPIED to host memory -- device chunks into reused pinned buffers, host (offloaded) chunks by
    memcpy -- so the engine may keep training while `write_dcp` runs on another thread; without it
    the chunks are views of the live buffers (a synchronous save)."""
    from .checkpoint import _writes_shards, _TPGeom, param_kind

    geo = _TPGeom(engine)
    write = _writes_shards(engine)
    skip = getattr(engine.module, "_dtg_ckpt_skip", set())
    tied = getattr(cfg, "tie_word_embeddings", False)
    tensors, mappings, fqns = [], {}, set()
    step = torch.tensor(float(engine.step_count))
    if write:
        keep = lambda n: n not in skip and not (geo.size > 1 and geo.rank != 0 and param_kind(n) == "rep")  # noqa: E731
        for hf, hshape, offs, sizes, views in _chunks(engine, cfg, keep):
            if hf == "lm_head.weight" and tied:
                continue
            if hf == "model.embed_tokens.weight" and tied:
                # an HF model with tied embeddings still lists `lm_head.weight` in its state dict
                # (not in its optimizer state): the reference's resume asks for that key
                tensors.append(("model.lm_head.weight", hshape, offs, views["p"]))
                mappings["model.lm_head.weight"] = ("model", "lm_head.weight")
            fqns.add(hf)
            for key, path, t in ((f"model.{hf}", ("model", hf), views["p"]),
                                 (f"optimizer.state.{hf}.exp_avg", ("optimizer", "state", hf, "exp_avg"), views["m"]),
                                 (f"optimizer.state.{hf}.exp_avg_sq", ("optimizer", "state", hf, "exp_avg_sq"),
                                  views["v"])):
                tensors.append((key, hshape, offs, t))
                mappings[key] = path
        for hf in sorted(fqns):  # one replicated 0-d "step" per parameter (deduplicated across ranks)
            key = f"optimizer.state.{hf}.step"
            tensors.append((key, [], [], step))
            mappings[key] = ("optimizer", "state", hf, "step")
    if host_pool is not None:
        tensors = host_pool.copy([(k, g, o, t) for k, g, o, t in tensors])
    multi = dist.is_initialized() and dist.get_world_size() > 1
    all_fqns = [None] * dist.get_world_size() if multi else [sorted(fqns)]
    if multi:
        dist.all_gather_object(all_fqns, sorted(fqns))
    rank0 = (dist.get_rank() if dist.is_initialized() else 0) == 0
    objects, meta = {}, None
    if rank0:
        names = sorted(set().union(*[set(x) for x in all_fqns]))
        group = dict(_adamw_group(optimizer), params=names)
        # one BYTE_IO item per field, under the keys torch's flatten_state_dict gives a one-group
        # AdamW state dict (`optimizer.param_groups.0.lr`, ...), so a stock `dcp.load` of
        # get_state_dict()'s optimizer state finds every key
        for k, v in group.items():
            key = f"optimizer.param_groups.0.{k}"
            objects[key] = v
            mappings[key] = ("optimizer", "param_groups", 0, k)
        meta = {"format": FORMAT, "step": int(engine.step_count), "global_step": global_step,
                "world_size": dist.get_world_size() if multi else 1, "tp_size": geo.size}
    return DcpSnapshot(tensors, objects, mappings, meta, multi)


def write_dcp(ckpt_dir, snap: DcpSnapshot, process_group=None):
    """Collective over `process_group` (default: the world): write a snapshot as the DCP tree
    (`.metadata` + one fsynced `__<rank>_0.distcp` per rank) plus dtg.json.  Issues collectives only
    on `process_group`, so with a dedicated gloo group it runs on a background thread while the
    training thread keeps the main group busy (--async-ckpt)."""
    import torch.distributed.checkpoint as dcp
    from torch.distributed.checkpoint import FileSystemWriter

    from .checkpoint import fsync_dir

    ckpt_dir = Path(ckpt_dir)
    ckpt_dir.mkdir(parents=True, exist_ok=True)
    SavePlanner, _ = _planners()
    writer = FileSystemWriter(str(ckpt_dir), single_file_per_rank=True, sync_files=True)
    dcp.save({}, storage_writer=writer, planner=SavePlanner(snap.tensors, snap.objects, snap.mappings),
             process_group=process_group, no_dist=not snap.multi)
    if snap.meta is not None:
        with open(ckpt_dir / META, "w") as fp:
            json.dump(snap.meta, fp)
            fp.flush()
            os.fsync(fp.fileno())
    if snap.multi:
        dist.barrier(group=process_group)
    fsync_dir(ckpt_dir)


def save_dcp(ckpt_dir, engine, optimizer, cfg, global_step=None):
    """Collective (every rank): write `ckpt_dir` as a DCP checkpoint of {"model": ...,
    "optimizer": ...} in the reference's layout (synchronous: chunks are read from the live
    buffers while DCP writes them)."""
    write_dcp(ckpt_dir, snapshot_dcp(engine, optimizer, cfg, global_step))


class HostPool:
    """Host copies of a save's chunks for --async-ckpt, in flat per-dtype buffers that are
    allocated once (page-locked, exact size: utils/pinned.py) and reused by every later save of
    the same layout.  Device chunks are copied with non_blocking copies and one device sync;
    host chunks (CPU-offloaded moments / master weights) by memcpy."""

    def __init__(self):
        self._bufs = {}  # dtype -> flat tensor

    def copy(self, items):
        from ..utils.pinned import pinned_zeros

        need = {}
        for _, _, _, t in items:
            if t.dim() > 0:
                need[t.dtype] = need.get(t.dtype, 0) + t.numel()
        for dt, n in need.items():
            if dt not in self._bufs or self._bufs[dt].numel() < n:
                self._bufs[dt] = None
                self._bufs[dt] = pinned_zeros(n, dt)
        pos = {dt: 0 for dt in need}
        out, dev = [], False
        for key, gshape, offs, t in items:
            if t.dim() == 0:
                out.append((key, gshape, offs, t.detach().to("cpu", copy=True)))
                continue
            n = t.numel()
            dst = self._bufs[t.dtype][pos[t.dtype]:pos[t.dtype] + n].view(t.shape)
            pos[t.dtype] += n
            dst.copy_(t.detach(), non_blocking=t.is_cuda)
            dev = dev or t.is_cuda
            out.append((key, gshape, offs, dst))
        if dev:
            torch.cuda.synchronize()
        return out


# ------------------------------------------------------------------------------ load
def load_dcp(ckpt_dir, engine, cfg, load_optimizer: bool = True) -> dict:
    """Collective: fill this rank's owned parameter (and AdamW-moment) slices from a DCP
    checkpoint written on any layout.  Returns the dtg.json record (step counters)."""
    import torch.distributed.checkpoint as dcp
    from torch.distributed.checkpoint import FileSystemReader

    ckpt_dir = Path(ckpt_dir)
    _, LoadPlanner = _planners()
    tied = getattr(cfg, "tie_word_embeddings", False)
    dests, first = [], None
    for hf, hshape, offs, sizes, views in _chunks(engine, cfg):
        if hf == "lm_head.weight" and tied:
            continue
        dests.append((f"model.{hf}", hshape, offs, views["p"]))
        if load_optimizer:
            dests.append((f"optimizer.state.{hf}.exp_avg", hshape, offs, views["m"]))
            dests.append((f"optimizer.state.{hf}.exp_avg_sq", hshape, offs, views["v"]))
        first = first or hf
    scalars = {}
    step = torch.zeros(())
    if load_optimizer and first is not None:
        scalars[f"optimizer.state.{first}.step"] = step
    multi = dist.is_initialized() and dist.get_world_size() > 1
    with torch.no_grad():
        dcp.load({}, storage_reader=FileSystemReader(str(ckpt_dir)), planner=LoadPlanner(dests, scalars),
                 no_dist=not multi)
    meta = {}
    if (ckpt_dir / META).exists():
        with open(ckpt_dir / META) as fp:
            meta = json.load(fp)
    if load_optimizer:
        engine.step_count = int(meta.get("step", int(step.item())))
    sync = getattr(engine, "sync_params_after_load", None)
    if sync is not None:
        sync()
    if multi:
        dist.barrier()
    return meta
