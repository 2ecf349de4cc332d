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
def test_dw_gemm_matches_f32(cuda, K, M, N, out_dtype):
    import dtg.ops  # noqa: F401

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
