"""HIP-graph captured training step (dtg.train.graph) == the eager loop, step for step."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _setup(name, dev):
    from dtg.models import build_model
    from dtg.parallel.data_parallel import DataParallel, FlatAdamW

    torch.manual_seed(0)
    model = build_model(name, device=dev)
    eng = DataParallel(model, mode="single")
    opt = FlatAdamW(eng, lr=1e-3)
    sched = torch.optim.lr_scheduler.CosineAnnealingLR(opt, T_max=10, eta_min=1e-4)
    return model, eng, opt, sched


@pytest.mark.parametrize("name", ["llama-tiny-d128", "gpt2-tiny"])
def test_graphed_step_matches_eager(cuda, name):
    from dtg.train.graph import GraphedStep

    g = torch.Generator().manual_seed(1)
    model, eng, opt, sched = _setup(name, cuda)
    V = model.config.vocab_size
    batches = [torch.randint(0, V, (2, 128), generator=g).to(cuda) for _ in range(7)]
    nv = 2 * 127
    if name.startswith("gpt2"):
        model.eval()  # dropout off: eager and replay draw different RNG offsets otherwise
    init = {n: p.detach().float().clone() for n, p in model.named_parameters()}
    ref_losses = []
    for b in batches:
        opt.zero_grad()
        out = model(input_ids=b, labels=b, num_valid=nv)
        eng.backward(out.loss)
        opt.step()
        sched.step()
        ref_losses.append(out.loss.item())
    ref = {n: p.detach().clone() for n, p in model.named_parameters()}

    model, eng, opt, sched = _setup(name, cuda)
    if name.startswith("gpt2"):
        model.eval()
    step = GraphedStep(model, eng, opt, sched, warmup=2, num_valid=nv)
    losses = [step({"input_ids": b, "labels": b}).item() for b in batches]
    assert step.graph is not None and step.steps == 7
    torch.cuda.synchronize()
    # hipBLASLt may pick other (equally valid) GEMM algorithms inside a capture, so the replayed
    # steps match the eager ones to rounding, not bitwise; a wrong step-dependent AdamW scalar
    # (lr, bias corrections) would move the loss and the weights far outside these bounds.
    for a, b in zip(losses, ref_losses):
        assert abs(a - b) <= 2e-3 * abs(b), (losses, ref_losses)
    # Compare the accumulated updates: Adam turns rounding-level gradient differences of
    # near-zero gradients into +-lr steps, so elementwise bounds are meaningless; a wrong lr or
    # bias correction would change the update norm by tens of percent.
    # (1-D parameters are skipped: GPT-2's key bias has an exactly-zero true gradient, so its
    # Adam updates are the sign of rounding noise in both runs.)
    for n, p in model.named_parameters():
        if p.dim() < 2:
            continue
        d_graph = p.detach().float() - init[n]
        d_eager = ref[n].float() - init[n]
        rel = ((d_graph - d_eager).norm() / d_eager.norm().clamp_min(1e-12)).item()
        assert rel < 0.05, (n, rel)


def test_adamw_device_hyper_matches_scalars(cuda):
    """The AdamW kernel reading [lr, 1-b1^t, sqrt(1-b2^t)] from device memory == scalar launch."""
    import math

    torch.manual_seed(0)
    n = 4096 + 8
    p0 = torch.randn(n, device=cuda).bfloat16()
    g = torch.randn(n, device=cuda).bfloat16()
    m0 = (0.1 * torch.randn(n, device=cuda)).bfloat16()
    v0 = (0.01 * torch.rand(n, device=cuda)).bfloat16()
    for step, lr in [(1, 1e-3), (7, 3e-4)]:
        a = [t.clone() for t in (p0, m0, v0)]
        b = [t.clone() for t in (p0, m0, v0)]
        torch.ops.dtg.adamw_(a[0], None, g, a[1], a[2], lr, 0.9, 0.999, 1e-8, 0.01, step, 0.5)
        hyper = torch.tensor([lr, 1 - 0.9 ** step, math.sqrt(1 - 0.999 ** step)], device=cuda)
        torch.ops.dtg.adamw_(b[0], None, g, b[1], b[2], 123.0, 0.9, 0.999, 1e-8, 0.01, 99, 0.5, hyper)
        for x, y in zip(a, b):
            assert torch.equal(x, y)


def test_chapter01_trainer_hip_graph(cuda, tmp_path):
    """Chapter 01 trainer with --hip-graph on: captured after 3 eager steps, replayed after."""
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, os.path.join(root, "01-single-gpu", "train_llm.py"), "-e", "hg", "-d", "synthetic",
           "-m", "llama-tiny-d128", "-s", "256", "-b", "2", "--num-samples", "64", "--save-dir", str(tmp_path),
           "--log-freq", "4", "--ckpt-freq", "1000", "--num-workers", "0", "--max-steps", "12", "--hip-graph", "on"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=os.path.join(root, "01-single-gpu"))
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-3000:]
    assert "HIP graph" in out
    recs = [json.loads(x) for x in (tmp_path / "hg" / "metrics-rank0.jsonl").read_text().splitlines()]
    assert len(recs) == 3 and all(x["running_loss"] == x["running_loss"] for x in recs)
    assert recs[-1]["time/backward"] == 0.0 and recs[-1]["global_step"] == 12


@pytest.mark.parametrize("attn_pdrop", [0.1, 0.0])
def test_graphed_gpt2_attention_dropout_redraws_every_replay(cuda, attn_pdrop):
    """GPT-2 in train mode under --hip-graph: the attention-dropout {seed, offset} comes from torch's
    CUDA generator as a device tensor (ops.philox_rng), so every replay of the captured step draws
    a new keep mask.  With lr = 0 the weights never move, so on one repeated batch the replayed
    losses differ only through the mask: all distinct with attn_pdrop > 0, all equal without it
    (residual / embedding dropout are off here, so nothing else is random)."""
    from dtg.models import build_model, resolve_config
    from dtg.parallel.data_parallel import DataParallel, FlatAdamW
    from dtg.train.graph import GraphedStep

    torch.manual_seed(0)
    cfg = resolve_config("gpt2-tiny", resid_pdrop=0.0, embd_pdrop=0.0, attn_pdrop=attn_pdrop)
    model = build_model(cfg, device=cuda)
    model.train()
    eng = DataParallel(model, mode="single")
    opt = FlatAdamW(eng, lr=0.0, weight_decay=0.0)
    b = torch.randint(0, cfg.vocab_size, (2, 128), generator=torch.Generator().manual_seed(3)).to(cuda)
    step = GraphedStep(model, eng, opt, None, warmup=2, num_valid=2 * 127)
    losses = [step({"input_ids": b, "labels": b}).item() for _ in range(6)]
    assert step.graph is not None
    replays = losses[2:]
    if attn_pdrop > 0:
        assert len(set(replays)) == len(replays), losses
    else:
        assert len(set(replays)) == 1, losses
