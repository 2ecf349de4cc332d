"""CP attention at the rime chapter's shape (1 x 8192 packed, Hq 24 / Hkv 8, D 128, cp 2) on
the synthetic:packed rows, 2 ranks sharing cuda:0 over gloo, vs the full varlen attention."""
import os, sys, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch
import dtg.ops  # noqa: F401
import dtg  # noqa
from _dist import run_distributed
S, HQ, HKV, D = 8192, 24, 8, 128

def rows(i):
    from dtg.data import SyntheticPacked, PackedCollator
    ds = SyntheticPacked(100, S, 156939, 156938, 512, 0)
    b = PackedCollator(156938)([ds[i]])
    return b

def tensors(seed):
    g = torch.Generator().manual_seed(seed)
    return [torch.randn(1, S, h, D, generator=g).bfloat16() for h in (HQ, HKV, HKV, HQ)]

def worker(rank, world, i):
    import dtg.ops  # noqa
    from dtg.parallel.context_parallel import cp_attention, cp_ranges, shard_zigzag, row_doc_starts
    torch.cuda.set_device(0); dev = torch.device("cuda:0")
    b = rows(i)
    docs = row_doc_starts(b["cu_seqlens"], 1, S)
    loc = [shard_zigzag(t, rank, world).to(dev) for t in tensors(i)]
    ql, kl, vl = (t.reshape(-1, *t.shape[2:]).clone().requires_grad_() for t in loc[:3])
    ranges = cp_ranges(rank, world, 1, S // (2 * world), dev, docs)
    o = cp_attention(ql, kl, vl, None, 1, ranges=ranges)
    o.backward(loc[3].reshape(-1, HQ, D))
    torch.cuda.synchronize()
    return [t.view(1, -1, *t.shape[1:]).detach().float().cpu() for t in (o, ql.grad, kl.grad, vl.grad)]

if __name__ == "__main__":
    from dtg.parallel.context_parallel import unshard_zigzag
    dev = torch.device("cuda:0")
    for i in range(int(sys.argv[1]) if len(sys.argv) > 1 else 4):
        b = rows(i)
        cu = b["cu_seqlens"].to(dev); mx = b["max_seqlen"]
        q, k, v, do = (t.to(dev) for t in tensors(i))
        qs, ks, vs = (t.reshape(S, *t.shape[2:]) for t in (q, k, v))
        o, lse = torch.ops.dtg.flash_attn_fwd(qs, ks, vs, cu, mx, D ** -0.5, True)
        grads = torch.ops.dtg.flash_attn_bwd(do.reshape(S, HQ, D), qs, ks, vs, o, lse, cu, mx, D ** -0.5, True)
        ref = [t.view(1, S, *t.shape[1:]).float().cpu() for t in (o,) + tuple(grads)]
        res = run_distributed(worker, 2, i)
        rec = {"row": i, "ndocs": len(cu) - 1, "min_doc": int((cu[1:] - cu[:-1]).min()), "max_doc": mx}
        for j, name in enumerate(("out", "dq", "dk", "dv")):
            got = unshard_zigzag([r[j] for r in res], 2)
            rec[name] = {"finite": bool(torch.isfinite(got).all()), "ref_finite": bool(torch.isfinite(ref[j]).all()),
                         "rel": float(((got - ref[j]).norm() / ref[j].norm()).item())}
        print(json.dumps(rec), flush=True)
