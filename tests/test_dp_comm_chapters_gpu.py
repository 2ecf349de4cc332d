"""Chapters 02 (ZeRO) and 04 (FSDP) through the trainer CLI with `--dp-comm xgmi-dma` (ZeRO /
FSDP collectives as copy-engine pulls over xGMI, parallel/xgmi_dp.py) against the same run with
the process group's collectives: 2 ranks sharing the box's one GPU (DTG_SHARED_DEVICE=1, gloo
as the process group), 4 steps of the tiny Llama; both runs exit 0 and log the same losses to
bf16 summation-order rounding."""
import os
import re
import subprocess
import sys

import pytest

from _dist import free_port

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(tmp_path, chapter, dp_comm):
    env = dict(os.environ, DTG_SHARED_DEVICE="1", DTG_XGMI_TIMEOUT="30")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), "train_llm.py",
           "-e", f"dpc_{dp_comm}", "-m", "llama-tiny-d128", "-b", "2", "-d", "synthetic", "--num-workers", "0",
           "--log-freq", "1", "--ckpt-freq", "1000", "--max-steps", "4", "--save-dir", str(tmp_path / dp_comm),
           "--dp-comm", dp_comm]
    r = subprocess.run(cmd, cwd=os.path.join(ROOT, chapter), env=env, capture_output=True, text=True, timeout=240)
    log = r.stdout + r.stderr
    assert r.returncode == 0, log[-3000:]
    # rank 0's per-step losses (both ranks log, and their lines interleave in any order)
    losses = [float(x) for x in re.findall(r"\[rank=0\][^\n]*'global_step': [1-9][0-9]*,[^\n]*'running_loss': ([0-9.eE+-]+)", log)]
    assert len(losses) >= 4, log[-3000:]
    return losses[:4], log


# chapter 02 over the copy engines trains through tests/test_transport_auto_gpu.py (its calibrated
# pick) and tests/test_xgmi_dp_gpu.py (ZeRO vs one process at 4 and 8 ranks)
@pytest.mark.parametrize("chapter", ["04-fully-sharded-data-parallel"])
def test_chapter_dp_comm_xgmi_dma_matches_process_group(tmp_path, chapter):
    ref, _ = _run(tmp_path, chapter, "rccl")
    got, log = _run(tmp_path, chapter, "xgmi-dma")
    assert "copy-engine pulls over xGMI" in log, log[-2000:]  # the engine reports the transport it used
    for a, b in zip(got, ref):
        assert abs(a - b) <= 2e-2 * abs(b), (got, ref)
