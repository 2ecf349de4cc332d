"""Weight-gradient GEMMs on a side stream (`DTG_DW_STREAM=1`, ops/grad_routing.py).

Every dW GEMM is issued on a second stream; the engines join it before a bucket / unit gradient
collective, at the end of each backward and so before the optimizer.  With a ~1 ms spin
enqueued on the side stream ahead of EVERY dW GEMM, a consumer that skipped the join would read
gradients the GEMM has not written yet: results must stay BIT-identical to the in-order run and
to the side-stream run without spins, for the single-device DP engine, DDP and ZeRO over a real
RCCL communicator (world of one, forced collectives) and FSDP.  The first version of this test
found a real race (profiles/r4/s12): GEMMs that read dY directly saw autograd's later in-place
accumulation of the residual gradient; only private (transposed-copy) operands go to the side
stream now.
"""
import pytest
import torch

from _dist import run_distributed

pytestmark = pytest.mark.gpu
MODEL = "llama-tiny-d128"
STEPS = 3
SPIN = 2_000_000


def _train(kind, side, force=False, accum=2, spin=True):
    from dtg.models import build_model, resolve_config
    from dtg.ops import functional as F_
    from dtg.ops import grad_routing as gr
    from dtg.parallel.data_parallel import DataParallel, FlatAdamW

    gr._DW_STREAM = side
    tn_min, F_._TN_MIN_TOKENS = F_._TN_MIN_TOKENS, 0  # the bench's TN path at this small token count
    calls = [0]
    real = gr.dw_stream
    if side:
        def spinning(device):
            s = real(device)
            if spin:
                s.wait_stream(torch.cuda.current_stream(device))
                with torch.cuda.stream(s):
                    torch.cuda._sleep(SPIN)
            calls[0] += 1
            return s

        gr.dw_stream = spinning
    try:
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
        g = torch.Generator().manual_seed(0)
        losses = []
        for _ in range(STEPS):
            ids = torch.randint(0, cfg.vocab_size, (4, 128), generator=g).to(dev)
            opt.zero_grad()
            for j, mb in enumerate(ids.chunk(accum)):
                ctx = eng.no_sync() if j < accum - 1 else torch.enable_grad()
                with ctx:
                    out = model(input_ids=mb, labels=mb)
                    eng.backward(out.loss)
            opt.step()
            losses.append(out.loss.item())
        if kind == "fsdp":
            sd = eng.full_state_dict(rank0_only=False)
            params = {k: v.cpu() for k, v in sd.items()}
        else:
            if hasattr(eng, "wait_param_gather"):
                eng.wait_param_gather()
            torch.cuda.synchronize()
            params = {n: p.detach().cpu().clone() for n, p in model.named_parameters()}
        return params, losses, calls[0]
    finally:
        gr._DW_STREAM = False
        gr.dw_stream = real
        F_._TN_MIN_TOKENS = tn_min


def _worker(rank, world, kind, spin):
    return _train(kind, True, force=True, spin=spin)


def _same(a, b):
    pa, la, _ = a
    pb, lb, _ = b
    assert la == lb, (la, lb)
    for n, v in pa.items():
        assert torch.equal(pb[n], v), n


@pytest.mark.parametrize("kind", ["single", "fsdp"])
def test_dw_side_stream_race_free(cuda, kind):
    """A spin ahead of every side-stream GEMM leaves the result bit-identical to the in-order run
    (a consumer that skipped the join would read unwritten gradients, an operand mutated on the
    main stream would be read late)."""
    torch.cuda.set_device(0)
    ref = _train(kind, False)
    fast = _train(kind, True, spin=False)
    slow = _train(kind, True, spin=True)
    assert slow[2] > 0
    _same(fast, slow)
    _same(ref, slow)


@pytest.mark.parametrize("kind", ["ddp", "zero"])
def test_dw_side_stream_rccl_engines_race_free(cuda, kind):
    torch.cuda.set_device(0)
    ref = _train("single", False)
    fast, = run_distributed(_worker, 1, kind, False, backend="nccl")
    slow, = run_distributed(_worker, 1, kind, True, backend="nccl")
    assert slow[2] > 0
    _same(fast, slow)
    _same(ref, slow)
