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
    assert (ck / ".metadata").exists() and (ck / "__0_0.distcp").exists() and (ck / "__1_0.distcp").exists()
    r = _torchrun("04-fully-sharded-data-parallel", base + ["--max-steps", "4"])
    out = r.stdout + r.stderr
    assert r.returncode == 0 and "Resuming" in out, out[-3000:]
    assert json.loads((tmp_path / "fs" / "state.json").read_text())["global_step"] == 4
