#!/usr/bin/env python3
"""The one-node 405B recipe (chapter 07's FSDP x TP with chapter 05's CPU offload) at EXACT
Llama-3.1-405B width with REAL collectives: W ranks share the one GPU (DTG_SHARED_DEVICE=1, gloo
between them), against a single-process oracle of the same width and depth.

Both runs load the same weights from one HF safetensors directory (models/loading.py: every rank
memory-maps the files and reads only its slices), so the 2-D layout and the oracle start from
identical parameters.  Each runs `--steps` optimizer steps on the same global batch sequence
(seeded synthetic tokens; data-parallel rank r takes rows [r*b, (r+1)*b)) and records, per step,
the global loss (mean over the data-parallel ranks' row losses) and, after the last step, a
fingerprint of every parameter in HF coordinates: sums and sums of squares in float64 of the
weights and of the 3-step update (weights minus the loaded ones) over the elements each rank owns
-- TP-replicated tensors counted once, FSDP shards disjoint -- summed over ranks.

    python tools/rehearse_405b_shared.py prep --dir /tmp/w405 --layers 2
    python tools/rehearse_405b_shared.py run --dir /tmp/w405 --layers 2 --tp 1 --batch 2 --out oracle.json
    DTG_SHARED_DEVICE=1 torchrun --nproc-per-node 4 tools/rehearse_405b_shared.py run --dir /tmp/w405 \\
        --layers 2 --tp 2 --batch 1 --out twod.json
    python tools/rehearse_405b_shared.py compare oracle.json twod.json

Reference: /root/reference/07-2d-parallel/train_llm.py:80-128, 05-training-llama-405b/train_llm.py:104-126.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

import dtg  # noqa: E402,F401

def _cfg(a):
    from dtg.models import resolve_config

    return resolve_config(a.model, num_hidden_layers=a.layers)


def _sync(device):
    if device.type == "cuda":
        torch.cuda.synchronize(device)


def prep(a):
    """Random bf16 weights of the reduced-depth model, written as HF safetensors shards."""
    from safetensors.torch import save_file

    from dtg.models import build_model
    from dtg.models.hf_compat import llama_to_hf

    cfg = _cfg(a)
    os.makedirs(a.dir, exist_ok=True)
    torch.manual_seed(0)
    t0 = time.perf_counter()
    model = build_model(cfg, device="cuda" if torch.cuda.is_available() else "cpu", dtype=torch.bfloat16)
    hf = llama_to_hf({k: v.detach() for k, v in model.state_dict().items()}, cfg)
    del model
    if cfg.tie_word_embeddings:  # HF checkpoints of tied models keep only the embedding
        hf.pop("lm_head.weight", None)
    shard, size, k = {}, 0, 0
    for name in sorted(hf):
        t = hf[name].to("cpu").contiguous()
        shard[name] = t
        size += t.numel() * t.element_size()
        if size > (4 << 30):
            save_file(shard, os.path.join(a.dir, f"model-{k:05d}.safetensors"))
            shard, size, k = {}, 0, k + 1
    if shard:
        save_file(shard, os.path.join(a.dir, f"model-{k:05d}.safetensors"))
    _drop_page_cache(a.dir)
    print(json.dumps({"prep_s": round(time.perf_counter() - t0, 1), "files": k + 1,
                      "params_B": round(sum(v.numel() for v in hf.values()) / 1e9, 3)}), flush=True)


def _drop_page_cache(d):
    """The written files' pages leave the page cache (it counts against the box's memory cap)."""
    for f in sorted(os.listdir(d)):
        fd = os.open(os.path.join(d, f), os.O_RDONLY)
        try:
            os.fsync(fd)
            os.posix_fadvise(fd, 0, 0, os.POSIX_FADV_DONTNEED)
        finally:
            os.close(fd)


def _owned_chunks(engine, cfg):
    """This rank's parameter chunks in HF coordinates, each element owned by exactly one rank
    (TP-replicated tensors on TP rank 0 only, FSDP shards disjoint): [(hf name, offsets, view)]."""
    from dtg.train.checkpoint import _TPGeom, _writes_shards, param_kind
    from dtg.train.dcp_ckpt import _chunks

    geo = _TPGeom(engine)
    if not _writes_shards(engine):
        return []
    keep = lambda n: not (geo.size > 1 and geo.rank != 0 and param_kind(n) == "rep")  # noqa: E731
    return [(hf, tuple(offs), views["p"]) for hf, hshape, offs, sizes, views in _chunks(engine, cfg, keep)]


def _fingerprint(chunks, initial, block=1 << 26):
    """{hf name: [sum w, sum w^2, sum d, sum d^2]} of the weights w and of the update d = w - w0,
    in float64, streamed in blocks where the weights live (the GPU: no host copies)."""
    out = {}
    for (hf, offs, view), w0 in zip(chunks, initial):
        s = out.setdefault(hf, [0.0, 0.0, 0.0, 0.0])
        wf, w0f = view.detach().reshape(-1), w0.reshape(-1)
        for i in range(0, wf.numel(), block):
            w = wf[i:i + block].double()
            d = w - w0f[i:i + block].to(w.device).double()
            s[0] += float(w.sum())
            s[1] += float((w * w).sum())
            s[2] += float(d.sum())
            s[3] += float((d * d).sum())
    return out


def run(a):
    import torch.distributed as dist

    from dtg.models import build_model
    from dtg.models.loading import load_pretrained
    from dtg.parallel.checkpointing import apply_activation_checkpointing
    from dtg.parallel.data_parallel import FlatAdamW
    from dtg.parallel.fsdp import FullyShard
    from dtg.parallel.tensor_parallel import make_mesh
    from dtg.utils.dist import init_distributed

    rank, _, world, device = init_distributed()
    cfg = _cfg(a)
    dp_group = tp_group = None
    dp_rank, dp = 0, 1
    if world > 1:
        dp_group, tp_group, dp_rank, _, dp = make_mesh(a.tp)
    with torch.device("meta"):
        model = build_model(cfg, tp_group=tp_group, init=False)
    apply_activation_checkpointing(model)
    t0 = time.perf_counter()
    eng = FullyShard(model, group=dp_group, tp_group=tp_group, policy="transformer", device=device,
                     cpu_offload=True, offload_params=False, grad_ring=4, seed=0)
    load_pretrained(eng, a.dir, cfg)
    opt = FlatAdamW(eng, lr=a.lr)
    build_s = time.perf_counter() - t0
    chunks = _owned_chunks(eng, cfg)
    initial = [v.detach().clone() for _, _, v in chunks]  # on the parameters' device (HBM, not host RAM)
    g = torch.Generator().manual_seed(1)
    rows = a.batch * dp
    batches = [torch.randint(0, cfg.vocab_size, (rows, a.seq), generator=g) for _ in range(a.steps)]
    losses, step_s = [], []
    for ids in batches:
        mine = ids[dp_rank * a.batch:(dp_rank + 1) * a.batch].to(device)
        _sync(device)
        t = time.perf_counter()
        opt.zero_grad()
        out = model(input_ids=mine, labels=mine)
        eng.backward(out.loss)
        opt.step()
        loss = out.loss.detach().float().cpu()
        _sync(device)
        step_s.append(round(time.perf_counter() - t, 2))
        if world > 1:
            dist.all_reduce(loss)  # every TP rank of a row holds the row's loss: mean over all ranks
            loss /= world
        losses.append(float(loss))
        if rank == 0:
            print(f"step {len(losses)} loss {losses[-1]:.6f} {step_s[-1]} s", flush=True)
    fp = _fingerprint(_owned_chunks(eng, cfg), initial)
    if world > 1:
        allfp = [None] * world
        dist.all_gather_object(allfp, fp)
        fp = {}
        for d in allfp:
            for k, v in d.items():
                t = fp.setdefault(k, [0.0, 0.0, 0.0, 0.0])
                for i in range(4):
                    t[i] += v[i]
    if rank == 0:
        rec = {"world": world, "tp": a.tp, "dp": dp, "batch_per_rank": a.batch, "seq": a.seq, "layers": a.layers,
               "losses": losses, "step_s": step_s, "build_load_s": round(build_s, 1),
               "peak_alloc_gb": round(torch.cuda.max_memory_allocated(device) / 1e9, 2) if device.type == "cuda" else None,
               "fingerprint": fp}
        with open(a.out, "w") as f:
            json.dump(rec, f)
        print(json.dumps({k: v for k, v in rec.items() if k != "fingerprint"}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def compare(a):
    """Losses per step, and per parameter the update's sum of squares (relative) and the weights'
    sum of squares (relative): all within bf16 tolerance."""
    o, t = (json.load(open(p)) for p in (a.oracle, a.twod))
    assert set(o["fingerprint"]) == set(t["fingerprint"]), "different parameter sets"
    worst_loss = max(abs(x - y) / abs(x) for x, y in zip(o["losses"], t["losses"]))
    worst_w = worst_d = 0.0
    worst_name = None
    for k, (s, q, ds, dq) in o["fingerprint"].items():
        s2, q2, ds2, dq2 = t["fingerprint"][k]
        worst_w = max(worst_w, abs(q2 - q) / max(q, 1e-30))
        r = abs(dq2 - dq) / max(dq, 1e-30)
        if r > worst_d:
            worst_d, worst_name = r, k
    ok = worst_loss < a.loss_tol and worst_w < a.fp_tol and worst_d < a.fp_tol
    print(json.dumps({"oracle_losses": o["losses"], "twod_losses": t["losses"], "worst_loss_rel": worst_loss,
                      "worst_weight_sumsq_rel": worst_w, "worst_update_sumsq_rel": worst_d,
                      "worst_update_param": worst_name, "n_params": len(o["fingerprint"]), "match": ok}), flush=True)
    return 0 if ok else 1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["prep", "run", "compare"])
    ap.add_argument("files", nargs="*")
    ap.add_argument("--model", default="meta-llama/Llama-3.1-405B")
    ap.add_argument("--dir", default="/tmp/w405")
    ap.add_argument("--layers", type=int, default=2)
    ap.add_argument("--tp", type=int, default=1)
    ap.add_argument("--batch", type=int, default=1, help="rows per data-parallel rank")
    ap.add_argument("--seq", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--lr", type=float, default=1e-4)
    ap.add_argument("--out", default="rehearsal.json")
    ap.add_argument("--loss-tol", type=float, default=1e-2)
    ap.add_argument("--fp-tol", type=float, default=3e-2)
    a = ap.parse_args()
    if a.mode == "prep":
        return prep(a)
    if a.mode == "run":
        return run(a)
    a.oracle, a.twod = a.files
    return compare(a)


if __name__ == "__main__":
    sys.exit(main())
