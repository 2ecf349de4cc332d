"""Direct-peer xGMI collectives (csrc/comm/xgmi.hip) vs the exact expected results.

Two processes share the one GPU of the test box: the IPC mapping, the signal/epoch barrier
protocol and the pull kernels run exactly as across GPUs (peer pointers are then local HBM,
so this checks the protocol and the arithmetic, not link bandwidth).  The bounded in-kernel
wait turns a protocol bug into a test failure instead of a hang.
"""
import pytest
import torch

from _dist import run_distributed

pytestmark = pytest.mark.gpu


def _worker(rank, world, engine="kernel"):
    import torch.distributed as dist

    from dtg.parallel.xgmi import XgmiCommunicator
    from dtg.utils import comm as dcomm

    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    c = XgmiCommunicator(None, capacity_bytes=8 << 20, device=dev, timeout_s=5.0, gather_engine=engine)
    out = {}
    for dtype in (torch.bfloat16, torch.float32):
        for n in (8, 4096, 1 << 20):
            if n * world * torch.tensor([], dtype=dtype).element_size() > c.capacity:
                continue
            g = torch.Generator().manual_seed(100 + n)
            full = [torch.randn(n * world, generator=g).to(dtype) for _ in range(world)]  # rank r's input
            mine = full[rank].to(dev)
            # all-gather of each rank's first n elements
            ag = torch.empty(n * world, dtype=dtype, device=dev)
            c.all_gather_into(ag, mine[:n].contiguous())
            # reduce-scatter of the full vectors
            rs = torch.empty(n, dtype=dtype, device=dev)
            c.reduce_scatter_into(rs, mine)
            ar = mine.clone()
            c.all_reduce_(ar)
            torch.cuda.synchronize()
            c.check()
            exp_ag = torch.cat([f[:n] for f in full])
            exp_sum = torch.stack([f.float() for f in full]).sum(0)
            out[(str(dtype), n)] = (
                torch.equal(ag.cpu(), exp_ag),
                (rs.cpu().float() - exp_sum[rank * n:(rank + 1) * n].to(dtype).float()).abs().max().item(),
                (ar.cpu().float() - exp_sum.to(dtype).float()).abs().max().item(),
            )
    # repeated back-to-back collectives (epoch protocol, buffer reuse)
    x = torch.full((4096,), float(rank + 1), device=dev)
    bad = torch.zeros((), device=dev)
    for i in range(50):
        y = x + i
        c.all_reduce_(y)
        bad += (y != world * (world + 1) / 2 + world * i).sum()
    torch.cuda.synchronize()
    c.check()
    out["repeat"] = bad.item()
    # routed through dtg.utils.comm (what tp_comm calls)
    dcomm.register_xgmi(None, c)
    y = dcomm.all_gather_dim0(torch.full((16, 64), float(rank), device=dev, dtype=torch.bfloat16), None)
    z = dcomm.reduce_scatter_dim0(torch.ones(32, 64, device=dev), None)
    torch.cuda.synchronize()
    out["routed"] = (y[:16].float().mean().item(), y[16:].float().mean().item(), z.mean().item(), tuple(z.shape))
    dcomm.unregister_xgmi(None)
    dist.barrier()
    c.close()
    return out


@pytest.mark.parametrize("engine", ["kernel", "dma"])
def test_xgmi_collectives_two_ranks(cuda, engine):
    """engine="dma": the all-gather's stage and pulls are copy-engine transfers (hipMemcpyAsync)."""
    res = run_distributed(_worker, 2, engine)
    for r in range(2):
        for k, v in res[r].items():
            if k == "repeat":
                assert v == 0, v
                continue
            if k == "routed":
                assert v[0] == 0.0 and v[1] == 1.0 and v[2] == 2.0 and v[3] == (16, 64), v
                continue
            ag_ok, rs_err, ar_err = v
            assert ag_ok, (r, k)
            tol = 0.05 if "bfloat16" in k[0] else 1e-5
            assert rs_err <= tol and ar_err <= tol, (r, k, rs_err, ar_err)
