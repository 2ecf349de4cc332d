"""Tensor + sequence parallel Llama (tp=2) on the GPU with its TP collectives on the direct-peer
xGMI library == the same model on one device (loss and every gradient).

Both ranks share the box's one GPU (see test_xgmi_gpu.py); the process group is gloo, used only
for the handle exchange and the loss head's MAX all-reduce -- every sequence all-gather /
reduce-scatter / TP all-reduce of the model runs through csrc/comm/xgmi.hip.
"""
import pytest
import torch

from _dist import run_distributed

pytestmark = pytest.mark.gpu
MODEL = "llama-tiny-d128"


def _ids(vocab, rows=2):
    g = torch.Generator().manual_seed(0)
    return torch.randint(0, vocab, (rows, 64), generator=g)


def _grads(model):
    return {n: p.main_grad.detach().float().cpu().clone() for n, p in model.named_parameters()}


def _run(model, eng, ids):
    eng.zero_grad()
    out = model(input_ids=ids, labels=ids)
    eng.backward(out.loss)
    return out.loss.item()


def _worker(rank, world, rows=2, chunks=1, engine="kernel", regather=False):
    import torch.distributed as dist

    from dtg.models import build_model, resolve_config
    from dtg.parallel.data_parallel import DataParallel
    from dtg.parallel.tensor_parallel import make_mesh, shard_full_state_dict
    from dtg.parallel.xgmi import XgmiCommunicator
    from dtg.utils import comm as dcomm

    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    _, tp_group, _, tp_rank, _ = make_mesh(2)
    dcomm.register_xgmi(tp_group, XgmiCommunicator(tp_group, capacity_bytes=16 << 20, device=dev, timeout_s=5.0,
                                                    gather_engine=engine))
    cfg = resolve_config(MODEL)
    torch.manual_seed(0)
    full = build_model(cfg, device="cpu", dtype=torch.bfloat16)
    model = build_model(cfg, device=dev, tp_group=tp_group, init=False)
    model.load_state_dict(shard_full_state_dict(full.state_dict(), cfg, tp_rank, 2))
    model.tp.overlap_chunks = chunks  # > 1: overlapped SP regions, xGMI collectives on a side stream
    model.tp.sp_regather = regather
    eng = DataParallel(model, mode="single", tp_group=tp_group, broadcast_from_rank0=False)
    loss = _run(model, eng, _ids(cfg.vocab_size, rows).to(dev))
    torch.cuda.synchronize()
    dcomm._XGMI[tp_group].check()
    res = (loss, _grads(model), tp_rank)
    dist.barrier()
    return res


@pytest.mark.parametrize("rows,chunks,engine", [(2, 1, "kernel"), (4, 2, "kernel"), (4, 2, "dma")])
def test_tp2_xgmi_matches_single_device(cuda, rows, chunks, engine):
    """chunks=2: overlapped regions whose row-parallel GEMMs write into the workspace slots
    (zero-copy reduce-scatter); engine="dma": copy-engine pulls on per-peer streams."""
    from dtg.models import build_model, resolve_config
    from dtg.parallel.data_parallel import DataParallel
    from dtg.parallel.tensor_parallel import unshard_state_dicts

    cfg = resolve_config(MODEL)
    torch.manual_seed(0)
    ref = build_model(cfg, device="cpu", dtype=torch.bfloat16).to(cuda)
    eng = DataParallel(ref, mode="single")
    ref_loss = _run(ref, eng, _ids(cfg.vocab_size, rows).to(cuda))
    ref_g = _grads(ref)
    res = run_distributed(_worker, 2, rows, chunks, engine)
    assert abs(res[0][0] - ref_loss) < 2e-2 * abs(ref_loss) and res[0][0] == res[1][0]
    shards = [r[1] for r in sorted(res, key=lambda r: r[2])]
    full = unshard_state_dicts(shards, cfg)
    for n, g in ref_g.items():
        rel = ((full[n] - g).norm() / g.norm().clamp_min(1e-12)).item()
        assert rel < 3e-2, (n, rel)


def _rel_diff(a, b):
    return max(((x - b[1][n]).norm() / b[1][n].norm().clamp_min(1e-12)).item() for n, x in a[1].items())


@pytest.mark.parametrize("rows,chunks,engine", [(2, 1, "kernel"), (4, 2, "kernel"), (4, 2, "dma")])
def test_tp2_xgmi_sp_regather_matches_kept(cuda, rows, chunks, engine):
    """--sp-regather on the xGMI transports: the backward re-gathers the column-parallel inputs
    (prefetched on the xGMI side stream); the loss is bitwise the kept-activation run's and every
    gradient agrees to bf16 rounding (the weight-gradient GEMM reads the same values from another
    buffer, and the BLAS kernel choice may follow the buffer; tools/diag_regather.py checks the
    re-gathered chunks equal the forward's bitwise)."""
    kept = run_distributed(_worker, 2, rows, chunks, engine, False)
    regathered = run_distributed(_worker, 2, rows, chunks, engine, True)
    for a, b in zip(kept, regathered):
        assert a[0] == b[0]
        assert _rel_diff(a, b) < 1e-2, _rel_diff(a, b)
