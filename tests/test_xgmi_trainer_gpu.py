"""Fail-loud xGMI in the training loop: chapter 06 (TP over the direct-peer library) with one
rank skipping a collective must exit NON-ZERO with the XgmiError in the log, instead of
training on stale data.  Two ranks share the box's one GPU (DTG_SHARED_DEVICE=1)."""
import os
import subprocess
import sys

import pytest

from _dist import free_port

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _launch(tmp_path, extra_env, tp_comm="xgmi"):
    env = dict(os.environ, DTG_SHARED_DEVICE="1", **extra_env)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), "train_llm.py",
           "-e", "xf", "-m", "llama-tiny-d128", "-b", "2", "-d", "synthetic", "--num-workers", "0",
           "--log-freq", "1", "--ckpt-freq", "1000", "--max-steps", "3", "--save-dir", str(tmp_path),
           "--tp-comm", tp_comm, "--tp-comm-mb", "8"]
    return subprocess.run(cmd, cwd=os.path.join(ROOT, "06-tensor-parallel"), env=env, capture_output=True, text=True,
                          timeout=240)


def test_ch06_xgmi_lost_peer_exits_nonzero(tmp_path):
    r = _launch(tmp_path, {"DTG_XGMI_FAULT": "1:5", "DTG_XGMI_TIMEOUT": "1"})
    log = r.stdout + r.stderr
    assert r.returncode != 0, log[-3000:]
    assert "xgmi barrier timed out" in log, log[-3000:]


def test_ch06_xgmi_healthy_run_exits_zero(tmp_path):
    r = _launch(tmp_path, {"DTG_XGMI_TIMEOUT": "20"}, tp_comm="xgmi-dma")
    log = r.stdout + r.stderr
    assert r.returncode == 0, log[-3000:]
    assert "'global_step': 3" in log, log[-3000:]
