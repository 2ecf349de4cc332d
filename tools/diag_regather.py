#!/usr/bin/env python3
"""Diagnostic for --sp-regather on the GPU (2 ranks sharing one GPU, TP collectives on the xGMI
library): one chunked MLP region, forward + backward with the gathered chunks kept and with them
re-gathered, in ONE process each, same inputs.  Prints whether the re-gathered chunks equal the
forward's gathered chunks bitwise and how far the weight gradients differ.

    DTG_SHARED_DEVICE=1 torchrun --nproc-per-node 2 tools/diag_regather.py [--engine kernel|dma]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

import dtg  # noqa: E402,F401


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--engine", default="kernel")
    ap.add_argument("--rows", type=int, default=256, help="local rows of the region input")
    ap.add_argument("--hidden", type=int, default=512)
    ap.add_argument("--inter", type=int, default=1024)
    ap.add_argument("--chunks", type=int, default=2)
    a = ap.parse_args()
    import torch.distributed as dist

    from dtg import ops
    from dtg.parallel import async_tp
    from dtg.parallel.xgmi import XgmiCommunicator
    from dtg.utils import comm as dcomm
    from dtg.utils.dist import init_distributed

    rank, _, world, dev = init_distributed()
    g = dist.new_group(list(range(world)))
    if a.engine != "none":
        dcomm.register_xgmi(g, XgmiCommunicator(g, capacity_bytes=64 << 20, device=dev, timeout_s=10.0,
                                                gather_engine=a.engine))
    torch.manual_seed(0)
    w_gu = (torch.randn(2 * a.inter // world, a.hidden, device=dev) * 0.05).bfloat16().requires_grad_(True)
    w_dn = (torch.randn(a.hidden, a.inter // world, device=dev) * 0.05).bfloat16().requires_grad_(True)
    torch.manual_seed(1 + rank)
    x = torch.randn(a.rows, a.hidden, device=dev).bfloat16().requires_grad_(True)
    dy = torch.randn(a.rows, a.hidden, device=dev).bfloat16()
    seen = {"fwd": [], "bwd": []}
    real_get = async_tp.RegatherHandle.get

    def spy_get(h):
        t = real_get(h)
        seen["bwd"].append(t.clone())
        return t

    async_tp.RegatherHandle.get = spy_get
    res = {}
    for regather in (False, True):
        seen["fwd"].clear()
        seen["bwd"].clear()
        for t in (w_gu, w_dn, x):
            t.grad = None

        def fn(xg, j, out=None):
            seen["fwd"].append(xg.detach().clone())
            return ops.swiglu_mlp(xg, w_gu, w_dn, out=out)

        y = async_tp.sp_region(x, fn, g, a.chunks, (w_gu, w_dn), regather=regather)
        y.backward(dy)
        if dev.type == "cuda":
            torch.cuda.synchronize()
        res[regather] = ([t.grad.clone() for t in (w_gu, w_dn, x)], [f.clone() for f in seen["fwd"]],
                         [b.clone() for b in seen["bwd"]])
    (gk, fk, _), (gr, fr, br) = res[False], res[True]
    same_chunks = len(br) == len(fr) and all(torch.equal(p, q) for p, q in zip(fr, br))
    diffs = [(p.float() - q.float()).abs().max().item() for p, q in zip(gk, gr)]
    if rank == 0:
        print({"engine": a.engine, "regathered_equals_forward_chunks": same_chunks, "n_regathered": len(br),
               "grad_max_abs_diff[w_gu, w_down, x]": diffs}, flush=True)
    dist.barrier()
    dist.destroy_process_group()




def model_main():
    """--model: the TP Llama (llama-tiny-d128) in one process, kept vs re-gathered per region kind
    (all / attention only / MLP only), every weight gradient compared bitwise."""
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", action="store_true")
    ap.add_argument("--engine", default="kernel")
    ap.add_argument("--rows", type=int, default=4)
    ap.add_argument("--chunks", type=int, default=2)
    a = ap.parse_args()
    import torch.distributed as dist

    from dtg.models import build_model, resolve_config
    from dtg.parallel import async_tp
    from dtg.parallel.data_parallel import DataParallel
    from dtg.parallel.tensor_parallel import make_mesh, shard_full_state_dict
    from dtg.parallel.xgmi import XgmiCommunicator
    from dtg.utils import comm as dcomm
    from dtg.utils.dist import init_distributed

    rank, _, world, dev = init_distributed()
    _, tp_group, _, tp_rank, _ = make_mesh(world)
    if a.engine != "none":
        dcomm.register_xgmi(tp_group, XgmiCommunicator(tp_group, capacity_bytes=16 << 20, device=dev, timeout_s=10.0,
                                                        gather_engine=a.engine))
    cfg = resolve_config("llama-tiny-d128")
    torch.manual_seed(0)
    full = build_model(cfg, device="cpu", dtype=torch.bfloat16)
    model = build_model(cfg, device=dev, tp_group=tp_group, init=False)
    model.load_state_dict(shard_full_state_dict(full.state_dict(), cfg, tp_rank, world))
    model.tp.overlap_chunks = a.chunks
    eng = DataParallel(model, mode="single", tp_group=tp_group, broadcast_from_rank0=False)
    g = torch.Generator().manual_seed(0)
    ids = torch.randint(0, cfg.vocab_size, (a.rows, 64), generator=g).to(dev)
    real_region = async_tp.sp_region
    out = {}
    for mode in ("kept", "all", "attn", "mlp", "kept2"):
        model.tp.sp_regather = mode not in ("kept", "kept2")

        def region(x, fn, grp, k, params, regather=False, _mode=mode):
            is_attn = len(params) > 2
            if _mode == "attn":
                regather = regather and is_attn
            elif _mode == "mlp":
                regather = regather and not is_attn
            return real_region(x, fn, grp, k, params, regather=regather)

        async_tp.sp_region = region
        eng.zero_grad()
        o = model(input_ids=ids, labels=ids)
        eng.backward(o.loss)
        if dev.type == "cuda":
            torch.cuda.synchronize()
        out[mode] = (o.loss.item(), {n: p.main_grad.detach().float().clone() for n, p in model.named_parameters()})
    if rank == 0:
        ref = out["kept"]
        for mode in ("kept2", "all", "attn", "mlp"):
            loss, gr = out[mode]
            bad = {n: (gr[n] - ref[1][n]).abs().max().item() for n in gr if not torch.equal(gr[n], ref[1][n])}
            print({"engine": a.engine, "mode": mode, "loss_equal": loss == ref[0], "differing": bad}, flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    model_main() if "--model" in sys.argv else main()
