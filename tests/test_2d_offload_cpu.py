"""Chapter 07's 2-D recipe with chapter 05's CPU offload: FSDP over dp x
tensor parallel over tp, with the gradients + AdamW state on the host (parameters on the host, or
resident with the host gradient ring).  On 4 gloo ranks (tp 2 x dp 2) every offload layout trains
to the same weights as the 2-D run without offload, and the offload layouts are bit-identical to
each other (the reference's 2-D script: /root/reference/07-2d-parallel/train_llm.py:45-52,80-128;
its offload: /root/reference/05-training-llama-405b/train_llm.py:104-126)."""
import pytest
import torch

from _dist import run_distributed

MODEL = "llama-tiny-d128"
TOL = dict(atol=3e-4, rtol=1e-3)


def _batches(vocab, n=3, rows=4, S=32):
    g = torch.Generator().manual_seed(0)
    return [torch.randint(0, vocab, (rows, S), generator=g) for _ in range(n)]


def _train_2d(rank, world, tp, configs):
    from dtg.models import build_model, resolve_config
    from dtg.parallel.data_parallel import FlatAdamW
    from dtg.parallel.fsdp import FullyShard
    from dtg.parallel.tensor_parallel import make_mesh

    dp_group, tp_group, dp_rank, tp_rank, dp = make_mesh(tp)
    cfg = resolve_config(MODEL)
    out = {}
    for offload, offload_params, ring in configs:
        with torch.device("meta"):
            model = build_model(cfg, tp_group=tp_group, init=False, dtype=torch.float32)
        eng = FullyShard(model, group=dp_group, tp_group=tp_group, device="cpu", seed=0, cpu_offload=offload,
                         offload_params=offload_params, grad_ring=ring, overlap_cpu_step=offload)
        opt = FlatAdamW(eng, lr=1e-2, eps=1e-3)
        sched = torch.optim.lr_scheduler.LambdaLR(opt, lambda s: 1.0 / (1 + s))
        losses = []
        for ids in _batches(cfg.vocab_size):
            per = ids.shape[0] // dp
            mine = ids[dp_rank * per:(dp_rank + 1) * per]
            opt.zero_grad()
            o = model(input_ids=mine, labels=mine)
            eng.backward(o.loss)
            opt.step()
            sched.step()
            losses.append(o.loss.item())
        out[(offload, offload_params, ring)] = (
            {k: v.clone() for k, v in eng.full_state_dict(rank0_only=False).items()}, losses, tp_rank)
    return out


@pytest.mark.slow
def test_2d_fsdp_tp_cpu_offload_matches_no_offload():
    configs = [(False, True, 0), (True, True, 0), (True, False, 0), (True, False, 2)]
    res = run_distributed(_train_2d, 4, 2, configs)
    for r in range(4):
        ref_sd, ref_losses, _ = res[r][(False, True, 0)]
        full_sd, full_losses, _ = res[r][(True, True, 0)]
        for n, t in ref_sd.items():  # host AdamW vs the device op: the same update to rounding
            torch.testing.assert_close(full_sd[n], t, **TOL, msg=f"rank {r} {n}")
        assert full_losses == pytest.approx(ref_losses, rel=1e-5)
        for c in ((True, False, 0), (True, False, 2)):  # resident parameters, with and without the ring
            sd, losses, _ = res[r][c]
            assert losses == full_losses, (c, r)
            for n, t in full_sd.items():
                assert torch.equal(sd[n], t), (c, r, n)
    # TP peers hold different shards of the same model; the dp replicas of a TP rank agree
    by_tp = {}
    for r in range(4):
        sd, _, tpr = res[r][(True, False, 2)]
        by_tp.setdefault(tpr, []).append(sd)
    for tpr, sds in by_tp.items():
        for n in sds[0]:
            assert torch.equal(sds[0][n], sds[1][n]), (tpr, n)


@pytest.mark.slow
def test_chapter07_cli_runs_with_cpu_offload(tmp_path):
    """`07-2d-parallel/train_llm.py --cpu-offload on` end to end (2 ranks, --tp 2): the engine logs
    the offload layout and the run trains."""
    import os
    import subprocess
    import sys

    from _dist import free_port

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.join(root, "07-2d-parallel", "train_llm.py"), "-e", "o7", "-d", "synthetic", "-m", MODEL,
           "-s", "32", "-b", "2", "--num-samples", "64", "--save-dir", str(tmp_path), "--log-freq", "1",
           "--ckpt-freq", "100", "--num-workers", "0", "--max-steps", "3", "--tp", "2", "--cpu-offload", "on",
           "--offload-params", "off"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=dict(os.environ, OMP_NUM_THREADS="1"))
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-3000:]
    assert "cpu offload: gradients and AdamW state on the host" in out, out[-3000:]
    assert "'global_step': 3" in out
