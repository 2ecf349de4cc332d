#!/usr/bin/env python3
"""Where does a DTG_FAKE_WORLD tensor-parallel rehearsal first produce a non-finite value?

    DTG_FAKE_WORLD=8 python tools/diag_fake_nan.py --tp 8 --steps 14 [--lr 0]

Builds bench.py's flagship job (Llama-3-8B, b16 x 1024 per TP group) as rank 0 of the fake
8-rank job and runs training steps.  Forward hooks on the embedding, every decoder layer and the
final norm record the first module whose output is non-finite, and the parameters are checked after
every update.  Output is one JSON line per step: loss, the max |activation| per layer, and the
first non-finite site.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tp", type=int, default=8)
    ap.add_argument("--steps", type=int, default=14)
    ap.add_argument("--lr", type=float, default=3e-5)
    ap.add_argument("--model", default="meta-llama/Meta-Llama-3-8B")
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--seq", type=int, default=1024)
    a = ap.parse_args()
    import torch
    import torch.distributed as dist
    from torch.testing._internal.distributed.fake_pg import FakeStore

    import bench
    import dtg  # noqa: F401
    import dtg.ops  # noqa: F401  (registers torch.ops.dtg before the wrappers below look them up)

    world = int(os.environ.get("DTG_FAKE_WORLD", "8"))
    os.environ.update(RANK="0", WORLD_SIZE=str(world), LOCAL_RANK="0", LOCAL_WORLD_SIZE=str(min(world, 8)))
    cuda = torch.cuda.is_available()
    device = torch.device("cuda:0" if cuda else "cpu")
    if cuda:
        torch.cuda.set_device(device)
    dist.init_process_group("fake", store=FakeStore(), rank=0, world_size=world)
    torch.manual_seed(0)
    args = argparse.Namespace(model=a.model, tp=a.tp, tp_comm="rccl", tp_overlap_chunks=2, parallel="zero",
                              bucket_mb=256, overlap_optimizer=0, dp_comm="rccl", lr=a.lr)
    # every collective helper reports whether its input / output is finite (first offender wins)
    from dtg.utils import comm

    coll = {}

    def wrap(name, out_of):
        fn = getattr(comm, name)

        def w(*xs, **kw):
            r = fn(*xs, **kw)
            if "first" not in coll:
                if cuda:
                    torch.cuda.synchronize()
                ins = [x for x in xs if torch.is_tensor(x)]
                out = out_of(r, xs)
                fin_in = all(bool(torch.isfinite(x).all()) for x in ins[1:] + ins[:1] if x is not out)
                fin_out = bool(torch.isfinite(out).all())
                coll["n"] = coll.get("n", 0) + 1
                if not fin_in or not fin_out:
                    coll["first"] = {"op": name, "call": coll["n"], "input_finite": fin_in, "output_finite": fin_out,
                                     "shape": list(out.shape)}
            return r
        setattr(comm, name, w)

    wrap("all_gather_dim0", lambda r, xs: r)
    wrap("reduce_scatter_dim0", lambda r, xs: r)
    wrap("all_reduce_", lambda r, xs: r)
    wrap("all_gather_dim0_into_async", lambda r, xs: xs[0])
    wrap("reduce_scatter_dim0_into_async", lambda r, xs: xs[0])
    # every native op reports the first call whose output is non-finite while its inputs are not
    kern = {}
    kcalls = {}
    OPS = ["add_rmsnorm_fwd", "rmsnorm_fwd", "rmsnorm_bwd", "swiglu_fwd", "swiglu_bwd", "swiglu_bwd_t",
           "flash_attn_fwd", "flash_attn_bwd", "flash_attn_bwd_qkv", "flash_attn_bwd_qkv_rope", "rope_",
           "transpose2d", "transpose_mats_", "ce_stats", "ce_grad_", "ce_fwd_bwd_", "embedding_bwd_"]

    def tensors(v):
        if torch.is_tensor(v):
            return [v]
        if isinstance(v, (tuple, list)):
            return [t for x in v for t in tensors(x)]
        return []

    def finite(ts):
        return all(bool(torch.isfinite(t).all()) for t in ts if t.is_floating_point() and t.numel())

    for op in OPS:
        try:
            orig = getattr(torch.ops.dtg, op)
        except (AttributeError, RuntimeError):
            continue

        def w(*xs, _orig=orig, _op=op, **kw):
            kcalls[_op] = kcalls.get(_op, 0) + 1
            if cuda:
                torch.cuda.synchronize()
            ins = tensors(list(xs))
            bad_in = [i for i, t in enumerate(ins) if t.is_floating_point() and t.numel() and not finite([t])]
            r = _orig(*xs, **kw)
            if "first" not in kern:
                if cuda:
                    torch.cuda.synchronize()
                outs = tensors(r) + ([xs[0]] if _op.endswith("_") else [])
                if not finite(outs):  # the first native op with a non-finite output, and its inputs
                    kern["first"] = {"op": _op, "shapes_in": [list(t.shape) for t in ins][:8],
                                     "strides_in": [list(t.stride()) for t in ins][:8],
                                     "nonfinite_inputs": bad_in, "after_collective_call": coll.get("n")}
                    if _op.startswith("flash_attn_bwd_qkv") and torch.is_tensor(r):
                        hq, hkv, d = xs[2], xs[3], xs[4]
                        reg = {"dq": r[:, : hq * d], "dk": r[:, hq * d:(hq + hkv) * d], "dv": r[:, (hq + hkv) * d:]}
                        info = {}
                        for k_, t_ in reg.items():
                            bad = ~torch.isfinite(t_.float())
                            rows = bad.any(1).nonzero().flatten()
                            info[k_] = {"n": int(bad.sum()), "rows": rows[:8].tolist(), "nrows": int(rows.numel())}
                        again = _orig(*xs, **kw)
                        if cuda:
                            torch.cuda.synchronize()
                        info["rerun_finite"] = finite(tensors(again))
                        info["rerun_equal_where_finite"] = bool(torch.equal(torch.nan_to_num(again.float()),
                                                                            torch.nan_to_num(r.float())))
                        kern["first"]["detail"] = info
                        if os.environ.get("DIAG_DUMP"):
                            torch.save({"args": [x.cpu() if torch.is_tensor(x) else x for x in xs]},
                                       os.environ["DIAG_DUMP"])
            return r
        setattr(torch.ops.dtg, op, w)
    # GEMMs (hipBLASLt through torch.mm / addmm; TunableOp picks the solution per shape)
    gemm = {}
    for gname in ("mm", "addmm"):
        gorig = getattr(torch, gname)

        def gw(*xs, _orig=gorig, _name=gname, **kw):
            r = _orig(*xs, **kw)
            if "first" not in gemm:
                if cuda:
                    torch.cuda.synchronize()
                ins = [x for x in xs if torch.is_tensor(x)]
                out = kw.get("out", r)
                if finite(ins) and not finite([out]):
                    gemm["first"] = {"op": _name, "shapes": [list(x.shape) for x in ins],
                                     "strides": [list(x.stride()) for x in ins], "out_shape": list(out.shape),
                                     "out_stride": list(out.stride()), "has_out": "out" in kw,
                                     "nonfinite": int((~torch.isfinite(out)).sum()), "after_collective_call": coll.get("n")}
            return r
        setattr(torch, gname, gw)
    job = bench.build_job(args, torch, device, cuda)
    model, engine, opt, cfg = job["model"], job["engine"], job["opt"], job["cfg"]
    first = {}
    amax = {}

    def fwd_hook(name):
        def hook(mod, inp, out):
            t = out[0] if isinstance(out, (tuple, list)) else out
            if not torch.is_tensor(t):
                return
            m = t.detach().float().abs().amax().item()
            amax[name] = m
            if not (m < float("inf")) and "fwd" not in first:
                first["fwd"] = name
        return hook

    mods = [("embed", model.embed_tokens)] + [(f"layer{i}", l) for i, l in enumerate(model.layers)]
    for name, m in mods:
        m.register_forward_hook(fwd_hook(name))
    batches = bench._batches(torch, cfg, a.batch, a.seq, a.steps, device, 7)
    for step, ids in enumerate(batches):
        first.clear()
        amax.clear()
        coll.clear()
        kern.clear()
        gemm.clear()
        kcalls.clear()
        opt.zero_grad()
        out = model(input_ids=ids, labels=ids, num_valid=a.batch * (a.seq - 1))
        loss = out.loss
        engine.backward(loss)
        if cuda:
            torch.cuda.synchronize()
        bad_grads = []
        for n, p in model.named_parameters():
            g = p.grad if getattr(p, "main_grad", None) is None else p.main_grad
            if g is not None and g.numel() and not bool(torch.isfinite(g).all()):
                bad_grads.append(f"{n}:{int((~torch.isfinite(g)).sum())}/{g.numel()}")
        opt.step()
        if cuda:
            torch.cuda.synchronize()
        bad_params = [n for n, p in model.named_parameters() if not torch.isfinite(p.detach()).all()]
        # the optimizer-written W^T copies the backward's dX GEMMs read (ops.functional._wt)
        wt_bad = []
        for n, p in model.named_parameters():
            ref = getattr(p, "_dtg_wt", None)
            if ref is None:
                continue
            t = ref[0].weight_t(ref[1])
            if t is None:
                continue
            if not torch.equal(t, p.detach().t()):
                d = (t.float() - p.detach().t().float())
                wt_bad.append(f"{n}:{int((d != 0).sum())}/{d.numel()} finite={bool(torch.isfinite(t).all())}")
        rec = {"step": step, "loss": float(loss.item()), "first_nonfinite_fwd": first.get("fwd"),
               "nonfinite_grads": bad_grads[:8], "n_nonfinite_grads": len(bad_grads),
               "first_nonfinite_collective": coll.get("first"), "collectives_checked": coll.get("n"),
               "first_kernel_with_nonfinite_output": kern.get("first"),
               "wt_mismatch": wt_bad[:6], "n_wt_mismatch": len(wt_bad), "first_gemm_nonfinite_from_finite": gemm.get("first"),
               "native_calls": dict(kcalls),
               "nonfinite_params_after_step": bad_params[:5], "n_nonfinite_params": len(bad_params),
               "amax": {k: (round(v, 2) if v < float("inf") else str(v)) for k, v in amax.items()
                        if k in ("embed", "layer0", "layer1", f"layer{len(model.layers) // 2}", f"layer{len(model.layers) - 1}")}}
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
