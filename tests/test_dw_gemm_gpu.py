"""Token-major weight-gradient GEMM (csrc/kernels/dw_gemm.hip) against an f32 PyTorch product:
c (=|+=) a^T @ b with a [K, M], b [K, N] bf16, output bf16 or f32, fresh and accumulating,
asymmetric operands (a transposed or swapped C write would fail), strided (non-contiguous row
pitch) operands, and the shape guard."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ref(a, b):
    return a.float().t() @ b.float()


@pytest.mark.parametrize("K,M,N", [(64, 256, 256), (1024, 512, 768), (4096, 1024, 256), (192, 2560, 512)])
@pytest.mark.parametrize("out_dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("variant", ["1", "2", "3", "4", "5"])
def test_dw_gemm_matches_f32(cuda, K, M, N, out_dtype, variant, monkeypatch):
    import dtg.ops  # noqa: F401

    monkeypatch.setenv("DTG_DWG_VARIANT", variant)

    g = torch.Generator(device="cuda").manual_seed(K + M + N)
    a = torch.randn(K, M, device="cuda", generator=g).to(torch.bfloat16)
    # asymmetric B: a per-column ramp, so a swapped C write cannot pass
    b = (torch.randn(K, N, device="cuda", generator=g) + torch.arange(N, device="cuda") / N).to(torch.bfloat16)
    ref = _ref(a, b)
    c = torch.full((M, N), float("nan"), device="cuda", dtype=out_dtype)
    torch.ops.dtg.dw_gemm_(a, b, c, False)
    tol = 1e-2 if out_dtype == torch.bfloat16 else 1e-4
    err = ((c.float() - ref).abs().max() / ref.abs().max()).item()
    assert err < tol, err
    c0 = torch.randn(M, N, device="cuda", generator=g).to(out_dtype)
    c1 = c0.clone()
    torch.ops.dtg.dw_gemm_(a, b, c1, True)
    ref1 = ref + c0.float()
    err = ((c1.float() - ref1).abs().max() / ref1.abs().max()).item()
    assert err < tol, err


def test_dw_gemm_strided_rows(cuda):
    import dtg.ops  # noqa: F401

    big_a = torch.randn(512, 1024 + 64, device="cuda").to(torch.bfloat16)
    big_b = torch.randn(512, 768 + 128, device="cuda").to(torch.bfloat16)
    a, b = big_a[:, 32:32 + 1024], big_b[:, 64:64 + 768]
    c = torch.empty(1024, 768, device="cuda", dtype=torch.bfloat16)
    torch.ops.dtg.dw_gemm_(a, b, c, False)
    ref = _ref(a, b)
    assert ((c.float() - ref).abs().max() / ref.abs().max()).item() < 1e-2


def test_dw_gemm_rejects_untiled_shapes(cuda):
    import dtg.ops  # noqa: F401

    a = torch.randn(64, 300, device="cuda").to(torch.bfloat16)
    b = torch.randn(64, 256, device="cuda").to(torch.bfloat16)
    c = torch.empty(300, 256, device="cuda", dtype=torch.bfloat16)
    with pytest.raises(RuntimeError, match="multiples of 256"):
        torch.ops.dtg.dw_gemm_(a, b, c, False)


def _train(hand, accum=2):
    from dtg.models import build_model, resolve_config
    from dtg.ops import functional as F_
    from dtg.parallel.data_parallel import DataParallel, FlatAdamW

    F_._DW_GEMM = hand
    real = F_.route_weight_grad_hand
    calls = [0]

    def counting(*a, **k):
        calls[0] += 1
        return real(*a, **k)

    F_.route_weight_grad_hand = counting
    try:
        cfg = resolve_config("llama-tiny-d128")
        torch.manual_seed(0)
        model = build_model(cfg, device=torch.device("cuda"))
        eng = DataParallel(model, mode="single")
        opt = FlatAdamW(eng, lr=1e-3)
        g = torch.Generator().manual_seed(0)
        losses = []
        for _ in range(3):
            ids = torch.randint(0, cfg.vocab_size, (8, 128), generator=g).cuda()
            opt.zero_grad()
            for j, mb in enumerate(ids.chunk(accum)):
                ctx = eng.no_sync() if j < accum - 1 else torch.enable_grad()
                with ctx:
                    out = model(input_ids=mb, labels=mb)
                    eng.backward(out.loss)
            opt.step()
            losses.append(out.loss.item())
        torch.cuda.synchronize()
        return {n: p.detach().float().cpu() for n, p in model.named_parameters()}, losses, calls[0]
    finally:
        F_._DW_GEMM = False
        F_.route_weight_grad_hand = real


def test_dw_gemm_in_llama_backward(cuda):
    """DTG_DW_GEMM path (hand dW GEMM + swiglu_bwd_h) trains like the hipBLASLt TN path:
    every projection's dW goes through the hand kernel, with gradient accumulation."""
    ref, ref_losses, n0 = _train(False)
    got, losses, n1 = _train(True)
    assert n0 == 0 and n1 > 0
    for a, b in zip(losses, ref_losses):
        assert abs(a - b) < 2e-2 * abs(b), (losses, ref_losses)
    for n, v in ref.items():
        rel = ((got[n] - v).norm() / v.norm().clamp_min(1e-12)).item()
        assert rel < 1e-2, (n, rel)
