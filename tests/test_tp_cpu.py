"""T2: tensor + sequence parallel (and 2-D dp x tp) on gloo == single-process Llama."""
import pytest
import torch

import dtg  # noqa: F401

from _dist import run_distributed
from test_engines_cpu import _batches, _train

TOL = dict(atol=3e-4, rtol=1e-3)


def _tp_worker(rank, world, tp, model_name, batches, engine_mode, chunks=None, regather=False):
    import torch.distributed as dist

    from dtg.models import build_model, resolve_config
    from dtg.parallel.data_parallel import DataParallel, FlatAdamW
    from dtg.parallel.tensor_parallel import make_mesh, shard_full_state_dict

    dp_group, tp_group, dp_rank, tp_rank, dp = make_mesh(tp)
    cfg = resolve_config(model_name)
    torch.manual_seed(0)
    full = build_model(cfg, device="cpu", dtype=torch.float32)
    model = build_model(cfg, device="cpu", dtype=torch.float32, tp_group=tp_group, init=False)
    model.load_state_dict(shard_full_state_dict(full.state_dict(), cfg, tp_rank, tp))
    calls = []
    model.tp.sp_regather = regather
    if chunks is not None:
        model.tp.overlap_chunks = chunks
        import dtg.parallel.async_tp as atp

        orig = atp.sp_region
        atp.sp_region = lambda x, fn, g, k, params, **kw: calls.append(k) or orig(x, fn, g, k, params, **kw)
    if engine_mode == "fsdp":
        from dtg.parallel.fsdp import FullyShard

        eng = FullyShard(model, group=dp_group, tp_group=tp_group, device="cpu")
    else:
        eng = DataParallel(model, mode=engine_mode if dp > 1 else "single", group=dp_group, tp_group=tp_group,
                           broadcast_from_rank0=False)
    opt = FlatAdamW(eng, lr=1e-2, eps=1e-3)
    losses = []
    for ids in batches:
        per = ids.shape[0] // dp
        mine = ids[dp_rank * per:(dp_rank + 1) * per]
        opt.zero_grad()
        out = model(input_ids=mine, labels=mine)
        eng.backward(out.loss)
        opt.step()
        losses.append(out.loss.item())
    if engine_mode == "fsdp":
        sd = eng.full_state_dict(rank0_only=False)
        return sd, losses, tp_rank, calls
    if hasattr(eng, "wait_param_gather"):
        eng.wait_param_gather()  # ZeRO leaves the last all-gather in flight until the next forward
    return {n: p.detach().clone() for n, p in model.named_parameters()}, losses, tp_rank, calls


@pytest.mark.parametrize("world,tp,mode,model_name", [(2, 2, "ddp", "llama-tiny-d128"), (4, 2, "zero", "llama-tiny-d128"),
                                                      (4, 2, "ddp", "llama-tiny-d128"), (4, 2, "fsdp", "llama-tiny-d128"),
                                                      (2, 1, "fsdp", "llama-tiny-d128"), (2, 2, "ddp", "qwen2-tiny"),
                                                      (4, 2, "fsdp", "qwen2-tiny")])
def test_tp_sp_matches_single(world, tp, mode, model_name):
    """llama-tiny-d128: tied embeddings + GQA (4 q / 2 kv heads), llama3 rope; qwen2-tiny adds
    the q/k/v biases (column-parallel, split like the weight's q / k / v row blocks)."""
    from dtg.models import resolve_config
    from dtg.parallel.tensor_parallel import unshard_state_dicts

    cfg = resolve_config(model_name)
    batches = _batches(cfg.vocab_size, 4, 32)
    ref, ref_losses = _train(model_name, "single", 0, 1, batches)
    res = run_distributed(_tp_worker, world, tp, model_name, batches, mode)
    shards = [r[0] for r in sorted(res[:tp], key=lambda r: r[2])]
    full = unshard_state_dicts(shards, cfg)
    for n in ref:
        torch.testing.assert_close(full[n], ref[n], **TOL, msg=n)
    # every dp replica identical
    for r in res[tp:]:
        for n, v in r[0].items():
            assert torch.equal(v, res[r[2]][0][n])


@pytest.mark.parametrize("chunks,mode", [(1, "ddp"), (4, "ddp"), (4, "fsdp")])
def test_tp_overlap_chunks_match_single(chunks, mode):
    """The overlapped SP regions (parallel/async_tp.py) at k = 4 chunks -- attention regions of
    one sequence per chunk, MLP regions of 16 rows -- and the synchronous path (k = 1) both
    train like the single-process model; engine notifications fire once per weight."""
    from dtg.models import resolve_config
    from dtg.parallel.tensor_parallel import unshard_state_dicts

    model_name = "llama-tiny-d128"
    cfg = resolve_config(model_name)
    batches = _batches(cfg.vocab_size, 8, 16)
    ref, ref_losses = _train(model_name, "single", 0, 1, batches)
    res = run_distributed(_tp_worker, 2, 2, model_name, batches, mode, chunks)
    # every layer ran both regions overlapped (k = 4), or none did (k = 1)
    assert res[0][3] == ([4] * (2 * cfg.num_hidden_layers * len(batches)) if chunks > 1 else []), res[0][3]
    for a, b in zip(res[0][1], ref_losses):
        assert abs(a - b) < 1e-4 * max(1.0, abs(b)), (res[0][1], ref_losses)
    shards = [r[0] for r in sorted(res, key=lambda r: r[2])]
    full = unshard_state_dicts(shards, cfg)
    for n in ref:
        torch.testing.assert_close(full[n], ref[n], **TOL, msg=n)


@pytest.mark.parametrize("chunks,mode", [(1, "ddp"), (4, "fsdp")])
def test_sp_regather_is_bitwise_the_kept_activations(chunks, mode):
    """--sp-regather: the column-parallel inputs re-gathered in the backward (synchronous
    sub-blocks at k = 1, overlapped regions at k = 4) train bit for bit like keeping them."""
    from dtg.models import resolve_config

    model_name = "llama-tiny-d128"
    cfg = resolve_config(model_name)
    batches = _batches(cfg.vocab_size, 8, 16)
    kept = run_distributed(_tp_worker, 2, 2, model_name, batches, mode, chunks, False)
    regathered = run_distributed(_tp_worker, 2, 2, model_name, batches, mode, chunks, True)
    for a, b in zip(kept, regathered):
        assert a[1] == b[1], (a[1], b[1])
        for n, v in a[0].items():
            assert torch.equal(v, b[0][n]), n


def test_regathered_swaps_only_the_gathered_tensor():
    """The saved-tensor hook replaces exactly the gathered activation (not the weight) and the
    backward's unpack re-gathers it (world 1: a copy of the local rows) -- once."""
    from dtg.parallel.async_tp import RegatherHandle, regathered

    local = torch.randn(8, 4)
    full = local.clone().requires_grad_(True)
    w = torch.randn(3, 4, requires_grad=True)
    with regathered(full, local, None) as h:
        y = torch.nn.functional.linear(full, w)
    assert isinstance(h, RegatherHandle) and h._buf is None  # nothing gathered yet
    gets = []
    real_get = h.get
    h.get = lambda: gets.append(real_get()) or gets[-1]
    y.sum().backward()
    assert len(gets) == 1 and torch.equal(gets[0], local)
    assert h._buf is None  # the handle does not keep the re-gathered rows past their use
    assert torch.allclose(w.grad, torch.ones(3, 8) @ local)
    assert torch.allclose(full.grad, torch.ones(8, 3) @ w)


def _init_worker(rank, world, engine):
    from dtg.models import build_model, resolve_config
    from dtg.parallel.tensor_parallel import make_mesh

    dp_group, tp_group, _, tp_rank, _ = make_mesh(world)
    cfg = resolve_config("llama-tiny")
    torch.manual_seed(0)
    if engine == "fsdp":
        from dtg.parallel.fsdp import FullyShard

        with torch.device("meta"):
            m = build_model(cfg, tp_group=tp_group, init=False, dtype=torch.float32)
        eng = FullyShard(m, group=dp_group, tp_group=tp_group, device="cpu", seed=0)
        sd = eng.full_state_dict(rank0_only=False)
    else:
        m = build_model(cfg, device="cpu", dtype=torch.float32, tp_group=tp_group)
        sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    return sd, tp_rank


@pytest.mark.parametrize("engine", ["ddp", "fsdp"])
def test_tp_random_init_differs_across_tp_ranks(engine):
    """Random init under TP: every sharded matrix gets different values on each TP rank (else
    the TP ranks' column / row blocks are copies that receive identical gradients forever);
    replicated norms stay identical."""
    res = run_distributed(_init_worker, 2, engine)
    (a, _), (b, _) = sorted(res, key=lambda r: r[1])
    for k in a:
        if k.endswith("layernorm.weight") or k == "norm.weight":
            assert torch.equal(a[k], b[k]), k
        else:
            assert not torch.equal(a[k], b[k]), k
            assert abs(a[k].std().item() - b[k].std().item()) < 0.2 * a[k].std().item(), k


def test_region_chunks():
    from dtg.parallel.async_tp import region_chunks

    assert region_chunks(64, 4) == 4 and region_chunks(64, 3) == 2 and region_chunks(63, 2) == 1
    assert region_chunks(2048, 4, 1024) == 2 and region_chunks(1024, 4, 1024) == 1
    assert region_chunks(100, 4, 64) == 1 and region_chunks(64, 1) == 1


def test_shard_unshard_roundtrip():
    from dtg.models import build_model, resolve_config
    from dtg.parallel.tensor_parallel import shard_full_state_dict, unshard_state_dicts

    cfg = resolve_config("llama-tiny")
    m = build_model(cfg, device="cpu", dtype=torch.float32)
    sd = m.state_dict()
    back = unshard_state_dicts([shard_full_state_dict(sd, cfg, r, 2) for r in range(2)], cfg)
    for k in sd:
        assert torch.equal(back[k], sd[k]), k


def _vp_ce_worker(rank, world, chunk, direct):
    import torch.distributed as dist

    import dtg.ops as ops
    from dtg.ops import grad_routing as gr

    g = torch.Generator().manual_seed(1)
    T, H, V = 64, 32, 48
    h = torch.randn(T, H, generator=g)
    w = torch.randn(V, H, generator=g) * 0.3
    lab = torch.randint(0, V, (T,), generator=g)
    lab[::7] = -100
    nv = int((lab != -100).sum())
    Vl = V // world
    wl = w[rank * Vl:(rank + 1) * Vl].clone().requires_grad_(True)
    hl = h.clone().requires_grad_(True)
    if direct:  # engine-owned loss: dW accumulates straight into main_grad
        wl.main_grad = torch.zeros_like(wl)
        gr.reset_grad_state([wl])
        gr.set_direct_loss_grad(True)
    loss = ops.vocab_parallel_fused_linear_cross_entropy(hl, wl, lab, rank * Vl, None, num_valid=nv, chunk=chunk)
    loss.backward()
    gr.set_direct_loss_grad(False)
    dh = hl.grad.clone()
    dist.all_reduce(dh)
    dw = wl.main_grad if direct else wl.grad
    return loss.item(), dh, dw.detach().clone()


@pytest.mark.parametrize("chunk,direct", [(16, False), (16, True), (64, False)])
def test_vocab_parallel_ce_pipelined_chunks_match_single(chunk, direct):
    """Vocab-parallel loss head with several chunks in flight (chunk j's stats all-gather
    overlapping chunk j+1's GEMM) == the single-process fused loss: loss, dh (summed over the
    TP ranks' partials) and each rank's dW shard."""
    import dtg.ops as ops

    g = torch.Generator().manual_seed(1)
    T, H, V = 64, 32, 48
    h = torch.randn(T, H, generator=g)
    w = (torch.randn(V, H, generator=g) * 0.3)
    lab = torch.randint(0, V, (T,), generator=g)
    lab[::7] = -100
    nv = int((lab != -100).sum())
    hr, wr = h.clone().requires_grad_(True), w.clone().requires_grad_(True)
    ref = ops.fused_linear_cross_entropy(hr, wr, lab, num_valid=nv, chunk=16)
    ref.backward()
    res = run_distributed(_vp_ce_worker, 2, chunk, direct)
    for r, (loss, dh, dw) in enumerate(res):
        assert abs(loss - ref.item()) < 1e-5, (loss, ref.item())
        torch.testing.assert_close(dh, hr.grad, atol=1e-5, rtol=1e-4)
        torch.testing.assert_close(dw, wr.grad[r * 24:(r + 1) * 24], atol=1e-5, rtol=1e-4)
