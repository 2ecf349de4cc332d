"""Flash attention must not read memory it did not write.  The caching allocator is poisoned
with NaN before each call, so `at::empty` workspaces (split dK / dV partials, delta) come back
full of NaN.  Every output must then be finite and bit-identical to the same call on a fresh
allocator.

Written while chasing the NaN of the DTG_FAKE_WORLD tensor-parallel rehearsals.  That turned out
to be upstream of attention (`profiles/r5/fake_nan/`).  The guard stays because the split dK / dV
path is the one place whose partials are `at::empty` buffers that several workgroups fill."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


def _poison(dev):
    """Fill freed allocator blocks of both pools with NaN (large: one 2 GiB block that later
    allocations are carved from; small: 2 MiB segments of sub-MiB tensors)."""
    torch.cuda.synchronize(dev)
    big = torch.full(((2 << 30) // 4,), float("nan"), dtype=torch.float32, device=dev)
    small = [torch.full((256 * 1024 // 4,), float("nan"), dtype=torch.float32, device=dev) for _ in range(64)]
    torch.cuda.synchronize(dev)
    del big, small


def _tables(max_pos, d, dev):
    inv = 1.0 / (10000.0 ** (torch.arange(0, d, 2, dtype=torch.float64) / d))
    f = torch.outer(torch.arange(max_pos, dtype=torch.float64), inv)
    return f.cos().float().contiguous().to(dev), f.sin().float().contiguous().to(dev)


@pytest.mark.parametrize("hq,hkv,nseq,S,rope", [
    (4, 1, 8, 1024, True),    # the TP = 8 rank of Llama-3-8B (split dK / dV, nsplit 4)
    (4, 1, 8, 1024, False),
    (8, 2, 4, 1024, True),    # TP = 4 (nsplit 2)
    (32, 8, 2, 1024, True),   # no split
])
def test_attention_backward_ignores_poisoned_workspaces(cuda, hq, hkv, nseq, S, rope):
    import dtg.ops  # noqa: F401

    ops = torch.ops.dtg
    D, T = 128, nseq * S
    g = torch.Generator(device=cuda).manual_seed(0)
    qkv = torch.randn(T, (hq + 2 * hkv) * D, device=cuda, generator=g).bfloat16()
    do = torch.randn(T, hq, D, device=cuda, generator=g).bfloat16()
    cu = torch.arange(0, T + 1, S, dtype=torch.int32, device=cuda)
    pos = torch.arange(S, device=cuda).repeat(nseq)
    cos, sin = _tables(S, D, cuda)
    scale = 1 / math.sqrt(D)
    q = qkv[:, : hq * D].view(T, hq, D)
    k = qkv[:, hq * D:(hq + hkv) * D].view(T, hkv, D)
    v = qkv[:, (hq + hkv) * D:].view(T, hkv, D)

    def run():
        o, lse = ops.flash_attn_fwd(q, k, v, cu, S, scale, True)
        if rope:
            d = ops.flash_attn_bwd_qkv_rope(do, qkv, hq, hkv, D, o, lse, cu, S, scale, True, cos, sin, pos)
        else:
            d = ops.flash_attn_bwd_qkv(do, qkv, hq, hkv, D, o, lse, cu, S, scale, True)
        torch.cuda.synchronize(cuda)
        return o.clone(), d.clone()

    torch.cuda.empty_cache()
    o_ref, d_ref = run()
    for trial in range(2):
        _poison(cuda)
        o, d = run()
        bad = {name: int((~torch.isfinite(t.float())).sum()) for name, t in
               (("o", o), ("dq", d[:, : hq * D]), ("dk", d[:, hq * D:(hq + hkv) * D]), ("dv", d[:, (hq + hkv) * D:]))}
        assert not any(bad.values()), (trial, bad)
        assert torch.equal(o, o_ref) and torch.equal(d, d_ref), trial
