"""Context-parallel attention on the gfx950 flash kernels (2 ranks sharing the box's GPU over
gloo) == the full-sequence flash attention, forward and backward (bf16 tolerances)."""
import pytest
import torch

from _dist import run_distributed

pytestmark = pytest.mark.gpu
S, HQ, HKV, D = 1024, 8, 2, 128


def _full(B):
    g = torch.Generator().manual_seed(0)
    return [torch.randn(B, S, h, D, generator=g).bfloat16() for h in (HQ, HKV, HKV, HQ)]


DOCS = [[0, 100, 333, 700], [0, 517]]  # packed rows: document starts per row


def _worker(rank, world, B, docs=None):
    import dtg.ops  # noqa: F401
    from dtg.parallel.context_parallel import cp_attention, cp_ranges, shard_zigzag

    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    loc = [shard_zigzag(t, rank, world).to(dev) for t in _full(B)]
    ql, kl, vl = (t.reshape(-1, *t.shape[2:]).clone().requires_grad_() for t in loc[:3])
    ranges = cp_ranges(rank, world, B, S // (2 * world), dev, docs) if docs else None
    o = cp_attention(ql, kl, vl, None, B, ranges=ranges)
    o.backward(loc[3].reshape(-1, HQ, D))
    torch.cuda.synchronize()
    return [t.view(B, -1, *t.shape[1:]).detach().float().cpu() for t in (o, ql.grad, kl.grad, vl.grad)]


@pytest.mark.parametrize("B", [1, 2])
@pytest.mark.parametrize("packed", [False, True])
def test_cp_attention_gpu_matches_full(cuda, packed, B):
    """Dense rows, and packed rows (documents cut across the zig-zag chunks) against the
    varlen flash attention over the full rows' documents.  B = 1 is the rime chapter's shape
    (one packed row: per-slot views of the LSE are not contiguous without a copy)."""
    import dtg.ops  # noqa: F401
    from dtg.parallel.context_parallel import unshard_zigzag

    q, k, v, do = (t.to(cuda) for t in _full(B))
    qs, ks, vs = (t.reshape(B * S, *t.shape[2:]) for t in (q, k, v))
    if packed:
        bounds = [b * S + d for b in range(B) for d in DOCS[b]] + [B * S]
        cu = torch.tensor(bounds, dtype=torch.int32, device=cuda)
        mx = max(int(x) for x in (cu[1:] - cu[:-1]).tolist())
    else:
        cu = torch.arange(0, (B + 1) * S, S, dtype=torch.int32, device=cuda)
        mx = S
    o, lse = torch.ops.dtg.flash_attn_fwd(qs, ks, vs, cu, mx, D ** -0.5, True)
    grads = torch.ops.dtg.flash_attn_bwd(do.reshape(B * S, HQ, D), qs, ks, vs, o, lse, cu, mx, D ** -0.5, True)
    ref = [t.view(B, S, *t.shape[1:]).float().cpu() for t in (o,) + tuple(grads)]
    res = run_distributed(_worker, 2, B, DOCS[:B] if packed else None)
    for i, name in enumerate(("out", "dq", "dk", "dv")):
        got = unshard_zigzag([r[i] for r in res], 2)
        rel = ((got - ref[i]).norm() / ref[i].norm()).item()
        assert rel < 2e-2, (name, rel)
