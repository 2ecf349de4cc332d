"""`--ac-layers auto` through chapter 05's trainer on the GPU (one process, FSDP at W = 1, CPU
offload off): the planner reads the caching allocator's peaks after the first steps, releases
layers within `--ac-budget-gb`, and the run trains exactly like the all-checkpointed one (same
per-step losses: checkpointing changes no value)."""
import json
import os
import re
import subprocess
import sys

import pytest

from _dist import free_port

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(tmp_path, tag, spec):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), "train_llm.py", "-e", tag, "-m", "llama-tiny-d128", "-b", "2", "-s", "256", "-d",
           "synthetic", "--num-workers", "0", "--log-freq", "1", "--ckpt-freq", "1000", "--max-steps", "5",
           "--save-dir", str(tmp_path), "--cpu-offload", "off", "--ac-layers", spec, "--ac-budget-gb", "100"]
    r = subprocess.run(cmd, cwd=os.path.join(ROOT, "05-training-llama-405b"), capture_output=True, text=True,
                       timeout=240, env=dict(os.environ, DTG_NO_WANDB="1"))
    log = r.stdout + r.stderr
    assert r.returncode == 0, log[-3000:]
    recs = [json.loads(x) for x in (tmp_path / tag / "metrics-rank0.jsonl").read_text().splitlines()]
    return recs, log


def test_ac_layers_auto_on_gpu_trains_like_all(cuda, tmp_path):
    ref, _ = _run(tmp_path, "all", "all")
    got, log = _run(tmp_path, "auto", "auto")
    plans = re.findall(r"--ac-layers auto \((\d)\): step-\d peak [0-9.]+ GB", log)
    assert plans[:2] == ["1", "2"], log[-3000:]  # planned from the caching allocator's peaks
    assert "no HBM to plan against" not in log
    assert [r["ac/layers"] for r in ref] == [2] * 5 and [r["ac/layers"] for r in got] == [0] * 5  # tiny: all fit
    # the recompute is the forward: same losses (tolerance only for atomics-ordered GPU reductions)
    assert [r["running_loss"] for r in got] == pytest.approx([r["running_loss"] for r in ref], rel=2e-3)
