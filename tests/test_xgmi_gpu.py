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
    out["routed"] = (y.view(world, 16, 64).float().mean((1, 2)).tolist(), z.mean().item(), tuple(z.shape))
    # zero-copy: the input is written straight into a workspace slot (no stage copy), twice per
    # slot so the slot-reuse wait is exercised; rows [r*8, (r+1)*8) of every rank's input sum up
    zc = []
    for i in range(4):
        buf = c.rs_input_buffer((8 * world, 64), torch.bfloat16, stage_bytes=8 * 64 * 2)
        assert buf is not None and c.ws.data_ptr() <= buf.data_ptr() < c.ws.data_ptr() + c.capacity
        buf.copy_(torch.full((8 * world, 64), float(rank + i), device=dev, dtype=torch.bfloat16))
        o = torch.empty(8, 64, device=dev, dtype=torch.bfloat16)
        w = dcomm.reduce_scatter_dim0_into_async(o, buf, None)
        w.wait()
        zc.append(o.float().mean().item())
    torch.cuda.synchronize()
    out["zero_copy"] = zc
    dcomm.unregister_xgmi(None)
    dist.barrier()
    c.close()
    return out


@pytest.mark.parametrize("engine,world", [("kernel", 2), ("dma", 2), ("kernel", 4), ("dma", 4)])
def test_xgmi_collectives(cuda, engine, world):
    """engine="dma": stage and pulls are copy-engine transfers (hipMemcpyAsync, one stream per
    peer); the reduce-scatter sums the pulled slices locally."""
    res = run_distributed(_worker, world, engine)
    for r in range(world):
        for k, v in res[r].items():
            if k == "repeat":
                assert v == 0, v
                continue
            if k == "zero_copy":
                exp = [sum(q + i for q in range(world)) for i in range(4)]
                assert v == exp, (r, v, exp)
                continue
            if k == "routed":
                assert v[0] == [float(q) for q in range(world)] and v[1] == float(world), v
                assert v[2] == (32 // world, 64), v
                continue
            ag_ok, rs_err, ar_err = v
            assert ag_ok, (r, k)
            tol = 0.05 if "bfloat16" in k[0] else 1e-5
            assert rs_err <= tol and ar_err <= tol, (r, k, rs_err, ar_err)


def _fault_worker(rank, world):
    import os
    import time

    import torch.distributed as dist

    from dtg.parallel.xgmi import XgmiCommunicator, XgmiError

    os.environ["DTG_XGMI_FAULT"] = "1:2"  # group rank 1 skips its third collective
    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    c = XgmiCommunicator(None, capacity_bytes=1 << 20, device=dev, timeout_s=0.5)
    x = torch.ones(1024, device=dev)
    t0 = time.time()
    for _ in range(20):  # after the first timeout every barrier returns at once (sticky error)
        c.all_reduce_(x)
    torch.cuda.synchronize()
    took = time.time() - t0
    err = None
    try:
        c.check()
    except XgmiError as e:
        err = str(e)
    dist.barrier()
    c.close()
    return err, took


def test_xgmi_barrier_timeout_is_sticky_and_raises(cuda):
    """A peer that skips a collective: the waiting rank's barrier times out once (not once per
    later collective), check() raises XgmiError naming the peer, nothing hangs."""
    res = run_distributed(_fault_worker, 2)
    err0, took0 = res[0]
    assert err0 is not None and "peer 1" in err0, res
    assert took0 < 10.0, took0  # one 0.5 s timeout, not 20 of them
