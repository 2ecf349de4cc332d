"""Host AdamW (FSDP CPU offload): the AVX-512, AVX2 and scalar paths of
csrc/cpu/adamw_host.h are bit-identical (one arithmetic definition with explicit FMAs; integer
round-to-nearest-even bf16 narrowing, so f32 denormals survive and NaNs stay NaN), and match an
f64 reference to bf16 rounding."""
import os

import pytest
import torch

import dtg  # noqa: F401
from dtg.ops import _native

pytestmark = pytest.mark.skipif(not _native.LOADED, reason="needs the native extension")


def _cpu_isas():
    flags = open("/proc/cpuinfo").read() if os.path.exists("/proc/cpuinfo") else ""
    out = ["scalar"]
    if " avx2 " in flags and " fma " in flags:
        out.append("avx2")
    if " avx512f " in flags:
        out.append("avx512")
    return out


def _inputs(n, dtype, edge):
    g = torch.Generator().manual_seed(n)
    p = torch.randn(n, generator=g)
    gr = torch.randn(n, generator=g)
    m = 0.1 * torch.randn(n, generator=g)
    v = 0.01 * torch.rand(n, generator=g)
    if edge:  # specials in every buffer at scattered positions
        sp = torch.tensor([float("nan"), float("inf"), -float("inf"), 0.0, -0.0, 1e-40, -3e-39, 1e38])
        for t in (p, gr, m):
            idx = torch.randint(0, n, (len(sp),), generator=g)
            t[idx] = sp
        v[torch.randint(0, n, (4,), generator=g)] = torch.tensor([0.0, 1e-40, float("inf"), float("nan")])
    return [t.to(dtype) for t in (p, gr, m, v)]


def _run(isa, bufs, step=3):
    os.environ["DTG_HOST_ADAMW_ISA"] = isa
    try:
        p, g, m, v = [t.clone() for t in bufs]
        torch.ops.dtg.adamw_cpu_(p, g, m, v, 1e-3, 0.9, 0.999, 1e-8, 0.01, step, 0.5)
        return p, m, v
    finally:
        os.environ.pop("DTG_HOST_ADAMW_ISA", None)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("n", [1, 15, 16, 17, 1000, 4099, 200_003])
@pytest.mark.parametrize("edge", [False, True])
def test_host_adamw_isa_paths_bit_identical(dtype, n, edge):
    bufs = _inputs(n, dtype, edge)
    ref = _run("scalar", bufs)
    for isa in _cpu_isas()[1:]:
        out = _run(isa, bufs)
        for a, b, name in zip(out, ref, "pmv"):
            assert torch.equal(a.view(torch.int16) if a.dtype == torch.bfloat16 else a.view(torch.int32),
                               b.view(torch.int16) if b.dtype == torch.bfloat16 else b.view(torch.int32)), (isa, name)


def test_host_adamw_matches_f64_reference():
    p, g, m, v = _inputs(100_000, torch.float32, False)
    out = _run(_cpu_isas()[-1], [p, g, m, v])
    step, lr, b1, b2, eps, wd, gs = 3, 1e-3, 0.9, 0.999, 1e-8, 0.01, 0.5
    pd, gd, md, vd = [t.double() for t in (p, g, m, v)]
    gd = gd * gs
    pd = pd * (1 - lr * wd)
    md = md + (gd - md) * (1 - b1)
    vd = vd * b2 + (1 - b2) * gd * gd
    pd = pd - lr / (1 - b1 ** step) * md / (vd.sqrt() / (1 - b2 ** step) ** 0.5 + eps)
    torch.testing.assert_close(out[0].double(), pd, atol=1e-6, rtol=1e-5)
    torch.testing.assert_close(out[1].double(), md, atol=1e-7, rtol=1e-5)
    torch.testing.assert_close(out[2].double(), vd, atol=1e-9, rtol=1e-4)  # (1 - b2) rounds to f32
