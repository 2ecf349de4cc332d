"""`--dp-comm auto` / `--tp-comm auto` through the trainer (parallel/transport.py): the startup
calibration times every transport on the job's group at its message size, verifies each against
the process group's result, logs the table and its pick -- and the run then trains exactly like
the same run with that transport named explicitly.  Two ranks share the box's one GPU
(DTG_SHARED_DEVICE=1, gloo process group; DTG_TRANSPORT_CALIBRATE=1 makes a gloo group
calibrate, which it otherwise skips as a rehearsal)."""
import os
import re
import subprocess
import sys

import pytest

from _dist import free_port

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(tmp_path, chapter, flag, value, tag):
    env = dict(os.environ, DTG_SHARED_DEVICE="1", DTG_XGMI_TIMEOUT="30", DTG_TRANSPORT_CALIBRATE="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), "train_llm.py",
           "-e", f"auto_{tag}", "-m", "llama-tiny-d128", "-b", "2", "-d", "synthetic", "--num-workers", "0",
           "--log-freq", "1", "--ckpt-freq", "1000", "--max-steps", "3", "--save-dir", str(tmp_path / tag),
           flag, value]
    r = subprocess.run(cmd, cwd=os.path.join(ROOT, chapter), env=env, capture_output=True, text=True, timeout=240)
    log = r.stdout + r.stderr
    assert r.returncode == 0, log[-3000:]
    # rank 0's per-step losses (both ranks log, and their lines interleave in any order)
    losses = [float(x) for x in re.findall(r"\[rank=0\][^\n]*'global_step': [1-9][0-9]*,[^\n]*'running_loss': ([0-9.eE+-]+)", log)]
    assert len(losses) >= 3, log[-3000:]
    return losses[:3], log


@pytest.mark.parametrize("chapter,flag,kind,names", [
    ("02-distributed-data-parallel", "--dp-comm", "dp", ("rccl", "xgmi-dma")),
    ("06-tensor-parallel", "--tp-comm", "tp", ("rccl", "xgmi", "xgmi-dma")),
])
def test_auto_transport_trains_like_its_pick(tmp_path, chapter, flag, kind, names):
    got, log = _run(tmp_path, chapter, flag, "auto", "auto")
    m = re.search(kind + r" transport calibration at [0-9.]+ MiB: (.*) -> ([a-z-]+)", log)
    assert m, log[-3000:]
    table, choice = m.group(1), m.group(2)
    for n in names:  # every candidate was timed and none disagreed with the process group
        assert re.search(rf"(^|, ){re.escape(n)} [0-9.]+ us", table), table
    assert "error" not in table and "differs" not in table, table
    assert choice in names
    ref, _ = _run(tmp_path, chapter, flag, choice, "explicit")
    assert got == ref, (choice, got, ref)
