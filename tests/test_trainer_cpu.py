"""Trainer end to end on CPU ranks (gloo): chapter 02 under torchrun with straggler timers,
chapter 04 (FSDP) sharded checkpoint + resume."""
import json
import os
import subprocess
import sys

import pytest

from _dist import free_port

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _torchrun(chapter_dir, args, nproc=2, timeout=400):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(nproc),
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.join(ROOT, chapter_dir, "train_llm.py")] + args
    env = dict(os.environ, OMP_NUM_THREADS="1")
    return subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env)


@pytest.mark.slow
def test_ddp_chapter_waiting_timers(tmp_path):
    r = _torchrun("02-distributed-data-parallel",
                  ["-e", "wt", "-d", "synthetic", "-m", "llama-tiny", "-s", "32", "--num-samples", "32",
                   "--save-dir", str(tmp_path), "--log-freq", "2", "--ckpt-freq", "100", "--num-workers", "0",
                   "--max-steps", "4", "--waiting-timers", "on"])
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-3000:]
    recs = [json.loads(line) for line in (tmp_path / "wt" / "metrics-rank0.jsonl").read_text().splitlines()]
    assert recs and all("time/waiting" in x for x in recs)
    assert abs(recs[-1]["time/total"] - sum(v for k, v in recs[-1].items()
                                            if k.startswith("time/") and k != "time/total")) < 1e-6


@pytest.mark.slow
def test_fsdp_chapter_checkpoint_resume(tmp_path):
    base = ["-e", "fs", "-d", "synthetic", "-m", "llama-tiny", "-s", "32", "--num-samples", "64",
            "--save-dir", str(tmp_path), "--log-freq", "1", "--ckpt-freq", "2", "--num-workers", "0",
            "--numel-to-wrap", "1000"]
    r = _torchrun("04-fully-sharded-data-parallel", base + ["--max-steps", "2"])
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    ck = tmp_path / "fs" / "checkpoint"
    # the reference's tree: torch DCP written by every rank (train/dcp_ckpt.py)
    assert (ck / ".metadata").exists() and (ck / "__0_0.distcp").exists() and (ck / "__1_0.distcp").exists()
    r = _torchrun("04-fully-sharded-data-parallel", base + ["--max-steps", "4"])
    out = r.stdout + r.stderr
    assert r.returncode == 0 and "Resuming" in out, out[-3000:]
    assert json.loads((tmp_path / "fs" / "state.json").read_text())["global_step"] == 4
    # the resumed steps continue the uninterrupted cosine schedule (the optimizer's lr is restored
    # from the scheduler: chainable schedulers compute the next lr from the group's current one)
    lrs = {json.loads(l)["global_step"]: json.loads(l)["lr"]
           for l in (tmp_path / "fs" / "metrics-rank0.jsonl").read_text().splitlines()}
    ref = tmp_path / "ref"
    r = _torchrun("04-fully-sharded-data-parallel", [a if a != str(tmp_path) else str(ref) for a in base]
                  + ["--max-steps", "4", "--ckpt-freq", "100"])
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    ref_lrs = {json.loads(l)["global_step"]: json.loads(l)["lr"]
               for l in (ref / "fs" / "metrics-rank0.jsonl").read_text().splitlines()}
    for step in (3, 4):
        assert lrs[step] == pytest.approx(ref_lrs[step], rel=1e-9), (step, lrs, ref_lrs)


@pytest.mark.slow
def test_fsdp_async_checkpoint_resume(tmp_path):
    """--async-ckpt: files are written on a background thread into .pending/ and published
    (state.json last) at the next save / end of training; a resumed run continues from it."""
    base = ["-e", "fa", "-d", "synthetic", "-m", "llama-tiny", "-s", "32", "--num-samples", "64",
            "--save-dir", str(tmp_path), "--log-freq", "1", "--ckpt-freq", "2", "--num-workers", "0",
            "--numel-to-wrap", "1000", "--async-ckpt", "on"]
    r = _torchrun("04-fully-sharded-data-parallel", base + ["--max-steps", "4"])
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    d = tmp_path / "fa"
    assert not (d / ".pending").exists()
    assert json.loads((d / "state.json").read_text())["global_step"] == 4
    # the reference's DCP tree, written on the writer thread over its own gloo group
    assert (d / "checkpoint" / ".metadata").exists() and (d / "rng.pt").exists() and (d / "lr_scheduler.pt").exists()
    r = _torchrun("04-fully-sharded-data-parallel", base + ["--max-steps", "6"])
    out = r.stdout + r.stderr
    assert r.returncode == 0 and "Resuming" in out, out[-3000:]
    assert json.loads((d / "state.json").read_text())["global_step"] == 6


def test_async_pending_save_is_not_a_checkpoint(tmp_path):
    """An async save that has not been finalized leaves no state.json behind."""
    import torch

    import dtg  # noqa: F401
    from dtg.models import build_model
    from dtg.parallel.data_parallel import DataParallel, FlatAdamW
    from dtg.train.checkpoint import CheckpointManager, has_checkpoint, new_state

    m = build_model("llama-tiny", device="cpu", dtype=torch.float32)
    eng = DataParallel(m, mode="single")
    opt = FlatAdamW(eng, lr=1e-3)
    sched = torch.optim.lr_scheduler.CosineAnnealingLR(opt, T_max=10)
    mgr = CheckpointManager(tmp_path, eng, opt, sched, "full", async_save=True)
    st = new_state()
    st["global_step"] = 3
    mgr.save(st)
    assert not has_checkpoint(tmp_path)
    mgr.finalize()
    assert has_checkpoint(tmp_path) and (tmp_path / "model.pt").exists() and not (tmp_path / ".pending").exists()
    assert json.loads((tmp_path / "state.json").read_text())["global_step"] == 3
    mgr2 = CheckpointManager(tmp_path, eng, opt, sched, "full")
    assert mgr2.load()["global_step"] == 3


def _losses(path):
    return [json.loads(line)["running_loss"] for line in path.read_text().splitlines()]


@pytest.mark.slow
@pytest.mark.parametrize("flag,dataset", [("--sp", "synthetic:packed"), ("--cp", "synthetic"),
                                          ("--cp", "synthetic:packed:20")])
def test_sequence_parallel_chapter_matches_single_process(tmp_path, flag, dataset):
    """rime chapter with each row split over 2 ranks (Ulysses on packed rows, context parallel on
    dense and packed rows) logs the same losses as one process reading the same batches."""
    base = ["-d", dataset, "-m", "llama-tiny-d128", "-s", "64", "--num-samples", "16", "--log-freq", "1",
            "--ckpt-freq", "100", "--num-workers", "0", "--max-steps", "3", "--lr", "1e-3"]
    one = _torchrun("00-rime", ["-e", "one", "--save-dir", str(tmp_path)] + base, nproc=1)
    assert one.returncode == 0, (one.stdout + one.stderr)[-3000:]
    two = _torchrun("00-rime", ["-e", "two", "--save-dir", str(tmp_path), flag, "2"] + base, nproc=2)
    assert two.returncode == 0, (two.stdout + two.stderr)[-3000:]
    a, b = _losses(tmp_path / "one" / "metrics-rank0.jsonl"), _losses(tmp_path / "two" / "metrics-rank0.jsonl")
    assert len(a) == len(b) == 3
    for x, y in zip(a, b):
        assert abs(x - y) < 2e-2 * abs(x), (a, b)


@pytest.mark.slow
def test_running_loss_window_means_match_per_step_losses(tmp_path):
    """The running loss is summed on the device and read only at log / checkpoint steps: a
    --log-freq 2 run with a checkpoint mid-window (--ckpt-freq 3) logs the pairwise means of the
    per-step losses of an otherwise identical --log-freq 1 run."""
    def run(name, log_freq, ckpt_freq):
        r = _torchrun("02-distributed-data-parallel",
                      ["-e", name, "-d", "synthetic", "-m", "llama-tiny", "-s", "32", "--num-samples", "64",
                       "--save-dir", str(tmp_path), "--log-freq", str(log_freq), "--ckpt-freq", str(ckpt_freq),
                       "--num-workers", "0", "--max-steps", "6"], nproc=1)
        assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
        return [json.loads(l)["running_loss"] for l in (tmp_path / name / "metrics-rank0.jsonl").read_text().splitlines()]

    per_step = run("l1", 1, 100)
    windows = run("l2", 2, 3)
    assert len(per_step) == 6 and len(windows) == 3
    for k in range(3):
        assert windows[k] == pytest.approx((per_step[2 * k] + per_step[2 * k + 1]) / 2, rel=1e-5)


@pytest.mark.slow
def test_pp_chapter_runs_and_checkpoint_reshards_to_no_pp(tmp_path):
    """Chapter 02 with --pp 2 (1F1B, gloo): trains, checkpoints with global layer names, and
    the checkpoint resumes under --pp 1 on 2 data-parallel ranks (stage layout -> DP layout)."""
    base = ["-e", "pp", "-d", "synthetic", "-m", "llama-tiny", "-s", "32", "--num-samples", "64", "-b", "4",
            "--save-dir", str(tmp_path), "--log-freq", "1", "--ckpt-freq", "2", "--num-workers", "0"]
    r = _torchrun("02-distributed-data-parallel", base + ["--max-steps", "2", "--pp", "2", "--pp-microbatches", "2"])
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-3000:]
    assert "pipeline stage 1/2" in out
    from torch.distributed.checkpoint import FileSystemReader

    names = set(FileSystemReader(str(tmp_path / "pp" / "checkpoint")).read_metadata().state_dict_metadata)
    assert {"model.model.layers.1.mlp.up_proj.weight", "model.model.layers.0.mlp.gate_proj.weight"} <= names
    r = _torchrun("02-distributed-data-parallel", base + ["--max-steps", "4"])
    out = r.stdout + r.stderr
    assert r.returncode == 0 and "Resuming" in out, out[-3000:]
    assert json.loads((tmp_path / "pp" / "state.json").read_text())["global_step"] == 4


def test_offload_grad_ring_auto_policy(monkeypatch):
    """--offload-grad-ring auto (profiles/r4/s23): on with the HBM-resident parameter layout, off
    with parameters on the host unless the node's host state would not fit in RAM, off under
    gradient accumulation."""
    import types

    import psutil
    import torch

    from dtg.train.trainer import _grad_ring_auto

    model = torch.nn.Linear(1000, 1000)  # 1.001 M parameters
    args = types.SimpleNamespace(grad_accum=1)
    assert _grad_ring_auto(args, model, None, offload_params=False) == 4
    assert _grad_ring_auto(args, model, None, offload_params=True) == 0  # plenty of host RAM
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "8")
    monkeypatch.setattr(psutil, "virtual_memory", lambda: types.SimpleNamespace(available=50_000_000))
    assert _grad_ring_auto(args, model, None, offload_params=True) == 4  # 8 ranks x 8 MB > 85 % of 50 MB
    args.grad_accum = 2
    assert _grad_ring_auto(args, model, None, offload_params=False) == 0


@pytest.mark.slow
def test_dp_comm_auto_child_crash_trains_on_rccl(tmp_path):
    """--dp-comm auto calibrates in a child job (parallel/transport.py resolve_isolated); a child
    that crashes leaves the trainer on RCCL (the process group), with the error logged, and the
    run trains to the end."""
    env_stub = json.dumps([sys.executable, "-c", "import sys; sys.stderr.write('boom'); sys.exit(7)"])
    os.environ["DTG_TRANSPORT_CHILD_CMD"] = env_stub
    try:
        r = _torchrun("02-distributed-data-parallel",
                      ["-e", "auto", "-d", "synthetic", "-m", "llama-tiny", "-s", "32", "--num-samples", "32",
                       "--save-dir", str(tmp_path), "--log-freq", "1", "--ckpt-freq", "100", "--num-workers", "0",
                       "--max-steps", "2", "--dp-comm", "auto"])
    finally:
        del os.environ["DTG_TRANSPORT_CHILD_CMD"]
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-3000:]
    assert "dp transport calibration" in out and "calibration child exited 7" in out and "-> rccl" in out, out[-3000:]
    recs = [json.loads(line) for line in (tmp_path / "auto" / "metrics-rank0.jsonl").read_text().splitlines()]
    assert len(recs) == 2
