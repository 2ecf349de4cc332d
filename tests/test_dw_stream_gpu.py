"""Weight-gradient GEMMs on a side stream (`DTG_DW_STREAM=1`, ops/grad_routing.py).

Every dW GEMM is issued on a second stream; the engines join it before a bucket / unit gradient
collective, at the end of each backward and so before the optimizer.  With a ~1 ms spin
enqueued on the side stream ahead of EVERY dW GEMM, a consumer that skipped the join would read
gradients the GEMM has not written yet: results must stay BIT-identical to the in-order run
(same GEMM kernels, same accumulation order), for the single-device DP engine, DDP and ZeRO over
a real RCCL communicator (world of one, forced collectives) and FSDP."""
import pytest
import torch

from _dist import run_distributed

pytestmark = pytest.mark.gpu
MODEL = "llama-tiny-d128"
STEPS = 3
SPIN = 2_000_000


def _train(kind, side, force=False, accum=2):
    from dtg.models import build_model, resolve_config
    from dtg.ops import grad_routing as gr
    from dtg.parallel.data_parallel import DataParallel, FlatAdamW

    gr._DW_STREAM = side
    calls = [0]
    if side:
        real = gr.dw_stream

        def spinning(device):
            s = real(device)
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
        if side:
            gr.dw_stream = real


def _worker(rank, world, kind, side):
    return _train(kind, side, force=True)


@pytest.mark.parametrize("kind", ["single", "fsdp"])
def test_dw_side_stream_bit_identical(cuda, kind):
    torch.cuda.set_device(0)
    ref, ref_losses, _ = _train(kind, False)
    got, losses, calls = _train(kind, True)
    assert calls > 0  # the side stream was used
    assert losses == ref_losses
    for n, v in ref.items():
        assert torch.equal(got[n], v), (kind, n)


@pytest.mark.parametrize("kind", ["ddp", "zero"])
def test_dw_side_stream_rccl_engines_bit_identical(cuda, kind):
    torch.cuda.set_device(0)
    ref, ref_losses, _ = _train("single", False)
    (got, losses, calls), = run_distributed(_worker, 1, kind, True, backend="nccl")
    assert calls > 0
    assert losses == ref_losses
    for n, v in ref.items():
        assert torch.equal(got[n], v), (kind, n)
