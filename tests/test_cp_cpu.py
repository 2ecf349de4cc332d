"""Context parallelism (zig-zag shards, all-gathered K/V, block-wise flash + lse merge) ==
full-sequence causal attention, forward and backward, on gloo ranks."""
import pytest
import torch

import dtg  # noqa: F401
import dtg.ops  # noqa: F401  (registers torch.ops.dtg)

from _dist import run_distributed

B, S, HQ, HKV, D = 2, 48, 4, 2, 16


def _full(seed=0):
    g = torch.Generator().manual_seed(seed)
    q = torch.randn(B, S, HQ, D, generator=g)
    k = torch.randn(B, S, HKV, D, generator=g)
    v = torch.randn(B, S, HKV, D, generator=g)
    do = torch.randn(B, S, HQ, D, generator=g)
    return q, k, v, do


def _reference():
    q, k, v, do = _full()
    qs, ks, vs = (t.reshape(B * S, *t.shape[2:]).requires_grad_() for t in (q, k, v))
    cu = torch.arange(0, (B + 1) * S, S, dtype=torch.int32)
    o, lse = torch.ops.dtg.flash_attn_fwd(qs, ks, vs, cu, S, D ** -0.5, True)
    dq, dk, dv = torch.ops.dtg.flash_attn_bwd(do.reshape(B * S, HQ, D), qs, ks, vs, o, lse, cu, S, D ** -0.5, True)
    return [t.view(B, S, *t.shape[1:]) for t in (o, dq, dk, dv)]


def _worker(rank, world):
    from dtg.parallel.context_parallel import cp_attention, shard_zigzag

    q, k, v, do = _full()
    loc = [shard_zigzag(t, rank, world) for t in (q, k, v, do)]
    ql, kl, vl = (t.reshape(-1, *t.shape[2:]).clone().requires_grad_() for t in loc[:3])
    o = cp_attention(ql, kl, vl, None, B)
    o.backward(loc[3].reshape(-1, HQ, D))
    return [t.view(B, -1, *t.shape[1:]).detach() for t in (o, ql.grad, kl.grad, vl.grad)]


@pytest.mark.parametrize("world", [1, 2, 3])
def test_cp_attention_matches_full(world):
    from dtg.parallel.context_parallel import unshard_zigzag

    ref = _reference()
    if world == 1:
        res = [_worker(0, 1)]
    else:
        res = run_distributed(_worker, world)
    for i, name in enumerate(("out", "dq", "dk", "dv")):
        got = unshard_zigzag([r[i] for r in res], world)
        torch.testing.assert_close(got, ref[i], atol=2e-5, rtol=2e-4, msg=name)


def test_zigzag_shard_roundtrip_and_batch():
    from dtg.parallel.context_parallel import cp_batch, shard_zigzag, unshard_zigzag

    x = torch.arange(2 * 24).view(2, 24)
    assert torch.equal(unshard_zigzag([shard_zigzag(x, r, 3) for r in range(3)], 3), x)
    ids, lab, pos, nv = cp_batch(x, 1, 3)
    assert nv == 2 * 23
    assert torch.equal(pos[0], torch.tensor([4, 5, 6, 7, 16, 17, 18, 19]))
    assert torch.equal(lab[0], torch.tensor([5, 6, 7, 8, 17, 18, 19, 20]))  # next token of the FULL row
    assert torch.equal(ids[0], pos[0])


def _train_cp(rank, world, steps_batches):
    from dtg.models import build_model
    from dtg.parallel.context_parallel import cp_batch
    from dtg.parallel.data_parallel import DataParallel, FlatAdamW

    torch.manual_seed(0)
    model = build_model("llama-tiny-d128", device="cpu", dtype=torch.float32,
                        cp_group=torch.distributed.group.WORLD if world > 1 else None)
    eng = DataParallel(model, mode="ddp" if world > 1 else "single", bucket_mb=1, grad_divisor=1)
    opt = FlatAdamW(eng, lr=1e-2, eps=1e-3)
    losses = []
    for ids in steps_batches:
        opt.zero_grad()
        if world > 1:
            x, lab, pos, nv = cp_batch(ids, rank, world)
            out = model(input_ids=x, labels=lab, position_ids=pos, num_valid=nv)
        else:
            out = model(input_ids=ids, labels=ids)
        eng.backward(out.loss)
        opt.step()
        losses.append(out.loss.item())
    return {n: p.detach().clone() for n, p in model.named_parameters()}, losses


@pytest.mark.parametrize("world", [2, 4])
def test_llama_context_parallel_training_matches_single(world):
    """Llama trained with context parallelism over `world` ranks == one process on full rows."""
    g = torch.Generator().manual_seed(3)
    batches = [torch.randint(0, 512, (2, 32), generator=g) for _ in range(2)]
    ref, ref_losses = _train_cp(0, 1, batches)
    res = run_distributed(_train_cp, world, batches)
    # each rank's loss is its share of the global mean
    assert abs(sum(r[1][0] for r in res) - ref_losses[0]) < 1e-4 * abs(ref_losses[0])
    for r in range(world):
        for n, v in ref.items():
            torch.testing.assert_close(res[r][0][n], v, atol=3e-4, rtol=1e-3, msg=f"rank {r} {n}")


def _packed_batches(n=2, B=2, S=32, eos=511):
    from dtg.data import PackedCollator

    g = torch.Generator().manual_seed(5)
    out = []
    for _ in range(n):
        rows = []
        for _ in range(B):
            x = torch.randint(0, eos, (S,), generator=g)
            cuts = torch.randint(1, S - 1, (3,), generator=g)  # three interior EOS: 4 documents
            x[cuts] = eos
            rows.append({"input_ids": x})
        out.append(PackedCollator(eos)(rows))
    return out


def _train_cp_packed(rank, world, batches):
    from dtg.models import build_model
    from dtg.parallel.context_parallel import cp_batch
    from dtg.parallel.data_parallel import DataParallel, FlatAdamW

    torch.manual_seed(0)
    model = build_model("llama-tiny-d128", device="cpu", dtype=torch.float32,
                        cp_group=torch.distributed.group.WORLD if world > 1 else None)
    eng = DataParallel(model, mode="ddp" if world > 1 else "single", bucket_mb=1, grad_divisor=1)
    opt = FlatAdamW(eng, lr=1e-2, eps=1e-3)
    losses = []
    for b in batches:
        opt.zero_grad()
        if world > 1:
            x, lab, pos, nv = cp_batch(b["input_ids"], rank, world, labels=b["labels"], position_ids=b["position_ids"])
            out = model(input_ids=x, labels=lab, position_ids=pos, cu_seqlens=b["cu_seqlens"], num_valid=nv)
        else:
            out = model(input_ids=b["input_ids"], labels=b["labels"], position_ids=b["position_ids"],
                        cu_seqlens=b["cu_seqlens"], max_seqlen=b["max_seqlen"])
        eng.backward(out.loss)
        opt.step()
        losses.append(out.loss.item())
    return {n: p.detach().clone() for n, p in model.named_parameters()}, losses


@pytest.mark.parametrize("world", [2, 4])
def test_llama_context_parallel_packed_rows_matches_single(world):
    """Packed rows (documents separated by EOS, positions restarting per document) under context
    parallelism == one process running the varlen packed path: local chunks are cut at document
    boundaries, each piece attends only its own document's prefix."""
    batches = _packed_batches()
    ref, ref_losses = _train_cp_packed(0, 1, batches)
    res = run_distributed(_train_cp_packed, world, batches)
    assert abs(sum(r[1][0] for r in res) - ref_losses[0]) < 1e-4 * abs(ref_losses[0])
    for r in range(world):
        for n, v in ref.items():
            torch.testing.assert_close(res[r][0][n], v, atol=3e-4, rtol=1e-3, msg=f"rank {r} {n}")


def test_packed_ranges_cut_chunks_at_documents():
    from dtg.parallel.context_parallel import packed_ranges

    # one row of 16 tokens, cp=2 -> chunks of 4: rank 0 holds chunks 0 and 3 ([0,4) and [12,16));
    # documents start at 0, 3 and 10
    cu, ks, kl, mq, mk = packed_ranges(0, 2, 1, 4, [[0, 3, 10]], "cpu")
    assert cu.tolist() == [0, 3, 4, 8]          # pieces [0,3) [3,4) | [12,16)
    assert ks.tolist() == [0, 3, 10] and kl.tolist() == [3, 1, 6] and (mq, mk) == (4, 6)
