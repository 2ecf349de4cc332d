"""The multi-GPU engine paths over a REAL RCCL communicator on the 1-GPU box.

RCCL refuses two ranks on one device, so the engines run in a world of one with
`force_collectives=True`: DDP's async bucket all-reduce, ZeRO's reduce-scatter into the grad
shard plus the in-place parameter all-gather left in flight into the next forward, and FSDP's
per-unit all-gather / reduce-scatter with storage `resize_(0)` of gathered buffers all run
through `ProcessGroupNCCL` work objects and their stream waits.  Results must be BIT-identical
to the collective-free single-device engine.

Delay injection: every async collective is issued from a side stream that first spins for
~`SPIN` GPU cycles (`torch.cuda._sleep`).  A consumer that reads a collective's output without
waiting on its work object then reads stale memory and the bitwise comparison fails."""
import pytest
import torch

from _dist import run_distributed

pytestmark = pytest.mark.gpu
MODEL = "llama-tiny-d128"
STEPS = 3
SPIN = 20_000_000  # ~10 ms at ~2 GHz


def _batches(vocab, S=128):
    g = torch.Generator().manual_seed(0)
    return [torch.randint(0, vocab, (4, S), generator=g) for _ in range(STEPS)]


def _install_delay():
    import torch.distributed as dist

    side = torch.cuda.Stream()

    def wrap(fn):
        def delayed(*a, **kw):
            if not kw.get("async_op", False):
                return fn(*a, **kw)
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                torch.cuda._sleep(SPIN)
                work = fn(*a, **kw)  # RCCL's stream waits for `side`, i.e. for the spin
            return work

        return delayed

    for name in ("all_reduce", "reduce_scatter_tensor", "all_gather_into_tensor"):
        setattr(dist, name, wrap(getattr(dist, name)))


def _train(kind, force, delay, accum=1, S=128, count_wt=False):
    from dtg.models import build_model, resolve_config
    from dtg.parallel.data_parallel import DataParallel, FlatAdamW

    dev = torch.device("cuda", torch.cuda.current_device())
    cfg = resolve_config(MODEL)
    torch.manual_seed(0)
    model = build_model(cfg, device=dev)
    if kind == "fsdp":
        from dtg.parallel.fsdp import FullyShard

        eng = FullyShard(model, device=dev, force_collectives=force)
    else:
        eng = DataParallel(model, mode=kind, bucket_mb=1, force_collectives=force)
    opt = FlatAdamW(eng, lr=1e-3)
    sched = torch.optim.lr_scheduler.LambdaLR(opt, lambda s: 1.0 / (1 + s))
    losses = []
    used = []
    if count_wt:  # which backward dX GEMMs got the engine's W^T copy instead of transposing
        import dtg.ops.functional as F_

        real = F_._wt

        def counting(w):
            ref = getattr(w, "_dtg_wt", None)
            used.append(ref is not None and ref[0].weight_t(ref[1]) is not None)
            return real(w)

        F_._wt = counting
    for ids in _batches(cfg.vocab_size, S):
        ids = ids.to(dev)
        opt.zero_grad()
        for j, mb in enumerate(ids.chunk(accum)):
            ctx = eng.no_sync() if j < accum - 1 else torch.enable_grad()
            with ctx:
                out = model(input_ids=mb, labels=mb)
                eng.backward(out.loss)
        opt.step()
        sched.step()
        losses.append(out.loss.item())
    mode = eng.mode
    if count_wt:
        F_._wt = real
        return used, losses, mode
    if kind == "fsdp":
        sd = eng.full_state_dict(rank0_only=False)
        return {k: v.cpu() for k, v in sd.items()}, losses, mode
    eng.wait_param_gather() if hasattr(eng, "wait_param_gather") else None
    torch.cuda.synchronize()
    return {n: p.detach().cpu().clone() for n, p in model.named_parameters()}, losses, mode


# (kind, delay, accum, S, count_wt): every world-1 RCCL configuration runs in ONE spawned process
# (process + communicator start-up dominated these tests); undelayed ones first, since the delay
# wraps torch.distributed's collectives for the rest of the process
_W1_CONFIGS = [("ddp", False, 1, 128, False), ("zero", False, 1, 128, False), ("fsdp", False, 1, 128, False),
               ("ddp", True, 1, 128, False), ("zero", True, 1, 128, False), ("fsdp", True, 1, 128, False),
               ("ddp", True, 2, 128, False), ("zero", True, 2, 128, False), ("zero", True, 1, 1024, False),
               ("zero", True, 1, 1024, True)]
_W1 = {}


def _world1_all(rank, world, configs):
    import gc

    out, delayed = {}, False
    for c in configs:
        kind, delay, accum, S, count_wt = c
        if delay and not delayed:
            _install_delay()
            delayed = True
        assert delay or not delayed, "undelayed configurations must come first"
        out[c] = _train(kind, True, delay, accum, S, count_wt)
        gc.collect()
        torch.cuda.empty_cache()
    return out


def _world1(kind, delay, accum, S=128, count_wt=False):
    if not _W1:
        (res,) = run_distributed(_world1_all, 1, _W1_CONFIGS, backend="nccl")
        _W1.update(res)
    return _W1[(kind, delay, accum, S, count_wt)]


def _single(kind, accum, S=128):
    torch.cuda.set_device(0)
    return _train("single" if kind != "fsdp" else "fsdp", False, False, accum, S)


@pytest.mark.parametrize("kind", ["ddp", "zero", "fsdp"])
@pytest.mark.parametrize("delay", [False, True])
def test_rccl_world1_engine_bit_identical(cuda, kind, delay):
    ref, ref_losses, ref_mode = _single(kind, 1)
    params, losses, mode = _world1(kind, delay, 1)
    assert mode == kind and ref_mode in ("single", "fsdp"), (mode, ref_mode)
    assert losses == ref_losses
    for n, v in ref.items():
        assert torch.equal(params[n], v), (kind, delay, n)


@pytest.mark.parametrize("kind", ["ddp", "zero"])
def test_rccl_world1_grad_accumulation(cuda, kind):
    ref, ref_losses, _ = _single(kind, 2)
    params, losses, mode = _world1(kind, True, 2)
    assert mode == kind and losses == ref_losses
    for n, v in ref.items():
        assert torch.equal(params[n], v), (kind, n)


def _offload_worker(rank, world, overlap, accum, offload_params=True, ring=0):
    from dtg.models import build_model, resolve_config
    from dtg.parallel.data_parallel import FlatAdamW
    from dtg.parallel.fsdp import FullyShard

    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    cfg = resolve_config(MODEL)
    torch.manual_seed(0)
    model = build_model(cfg, device=dev)
    eng = FullyShard(model, device=dev, cpu_offload=True, overlap_cpu_step=overlap, offload_params=offload_params,
                     grad_ring=ring)
    opt = FlatAdamW(eng, lr=1e-3)
    sched = torch.optim.lr_scheduler.LambdaLR(opt, lambda s: 1.0 / (1 + s))  # lr changes every step
    stepped = []
    for ids in _batches(cfg.vocab_size):
        per = ids.shape[0] // world
        mine = ids[rank * per:(rank + 1) * per].to(dev)
        opt.zero_grad()
        for j, mb in enumerate(mine.chunk(accum)):
            ctx = eng.no_sync() if j < accum - 1 else torch.enable_grad()
            with ctx:
                eng.backward(model(input_ids=mb, labels=mb).loss)
        stepped.append(eng._bwd_stepped)
        opt.step()
        sched.step()
    return {k: v.cpu() for k, v in eng.full_state_dict(rank0_only=False).items()}, stepped


def _offload_configs(rank, world, configs):
    """Every offload configuration in ONE spawn of the ranks (process start-up dominates)."""
    import gc

    out = {}
    for c in configs:
        out[c] = _offload_worker(rank, world, *c)
        gc.collect()
        torch.cuda.empty_cache()
    return out


# (overlap, accum, offload_params, ring)
_OFFLOAD_CONFIGS = [(True, 1, True, 0), (False, 1, True, 0), (True, 2, True, 0), (False, 2, True, 0),
                    (True, 1, False, 0), (True, 2, False, 0), (False, 1, False, 0),
                    (True, 1, False, 4), (True, 1, False, 1), (True, 1, True, 2)]
_OFFLOAD = {}


def _offload_results():
    if not _OFFLOAD:
        res = run_distributed(_offload_configs, 2, _OFFLOAD_CONFIGS)
        _OFFLOAD.update({c: [res[r][c] for r in range(2)] for c in _OFFLOAD_CONFIGS})
    return _OFFLOAD


def _same(a, b, tag):
    for r in range(2):
        for n, t in b[r][0].items():
            assert torch.equal(a[r][0][n], t), (tag, r, n)


@pytest.mark.parametrize("accum", [1, 2])
def test_fsdp_cpu_offload_overlap_bit_identical_on_gpu(cuda, accum):
    """pinned host shards, non_blocking H2D gathers, reduce-scatter -> D2H and the
    host-AdamW worker thread running while GPU streams are live: overlapped == post-backward."""
    res = _offload_results()
    on, off = res[(True, accum, True, 0)], res[(False, accum, True, 0)]
    for r in range(2):
        assert all(on[r][1]) and not any(off[r][1])
    _same(on, off, ("overlap", accum))


@pytest.mark.parametrize("overlap,accum", [(True, 1), (True, 2), (False, 1)])
def test_fsdp_resident_param_offload_bit_identical_on_gpu(cuda, overlap, accum):
    """offload_params=False: shards resident in HBM, host AdamW from the worker thread copying
    each updated unit back on the H2D side stream while backward kernels are still running; the
    next forward's gathers wait on those copies == the full offload, bit for bit."""
    res = _offload_results()
    _same(res[(overlap, accum, False, 0)], res[(overlap, accum, True, 0)], ("resident", overlap, accum))


def test_rccl_world1_zero_weight_t_with_delayed_gathers(cuda):
    """ZeRO's W^T copies are rebuilt per bucket on a side stream after the bucket's parameter
    all-gather lands (parallel/data_parallel.py).  With every all-gather delayed ~10 ms on the
    GPU, a transpose that did not wait for its gather would copy the pre-update weights and the
    dX GEMMs would use them: training must stay bit-identical to the single-device engine (whose
    copies the optimizer kernel writes), and every backward dX GEMM at >= 4096 tokens must use
    a copy (no per-weight transposes in the backward)."""
    ref, ref_losses, _ = _single("zero", 1, S=1024)
    params, losses, mode = _world1("zero", True, 1, 1024)
    assert mode == "zero" and losses == ref_losses
    for n, v in ref.items():
        assert torch.equal(params[n], v), n
    used, _, _ = _world1("zero", True, 1, 1024, True)
    assert used and all(used), f"{used.count(False)} of {len(used)} dX GEMMs transposed W in the backward"


@pytest.mark.parametrize("offload_params,ring", [(False, 4), (False, 1), (True, 2)])
def test_fsdp_offload_grad_ring_bit_identical_on_gpu(cuda, offload_params, ring):
    """Host gradient ring on the GPU: each unit's reduced gradient is copied D2H on the side
    stream into a reused pinned slot while the host AdamW of earlier units reads other slots
    (one slot: every D2H waits for the previous unit's host update) == the whole-model host
    gradient shard, bit for bit."""
    res = _offload_results()
    got, full = res[(True, 1, offload_params, ring)], res[(True, 1, offload_params, 0)]
    for r in range(2):
        assert all(got[r][1])
    _same(got, full, ("ring", offload_params, ring))
