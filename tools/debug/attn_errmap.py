"""Debug helper: where do flash-attention outputs differ from the f32 reference?"""
import math
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import dtg  # noqa
import dtg.ops  # noqa

dops = torch.ops.dtg
dev = torch.device("cuda:0")
for causal in (False, True):
    for (T, hq, hkv, D) in ((128, 1, 1, 128), (256, 2, 1, 128), (64, 1, 1, 64)):
        torch.manual_seed(0)
        q = torch.randn(T, hq, D).bfloat16(); k = torch.randn(T, hkv, D).bfloat16(); v = torch.randn(T, hkv, D).bfloat16()
        cu = torch.tensor([0, T], dtype=torch.int32)
        o_ref, lse_ref = dops.flash_attn_fwd(q, k, v, cu, T, 1 / math.sqrt(D), causal)
        o, lse = dops.flash_attn_fwd(q.to(dev), k.to(dev), v.to(dev), cu.to(dev), T, 1 / math.sqrt(D), causal)
        err = (o.float().cpu() - o_ref.float()).abs()
        lerr = (lse.cpu() - lse_ref).abs()
        print(f"causal={causal} T={T} hq={hq} hkv={hkv} D={D}: max o err {err.max():.3g}, max lse err {lerr.max():.3g}")
        if err.max() > 0.05:
            e_q = err.amax(dim=(1, 2))
            e_d = err.amax(dim=(0, 1))
            print("  err by q (first 64):", [round(x, 2) for x in e_q[:64].tolist()])
            print("  err by d:", [round(x, 2) for x in e_d.tolist()])
            print("  lse err by q (first 40):", [round(x, 3) for x in lerr[0, :40].tolist()])
        # v = identity-ish check: V[key][d] = (key == d)
