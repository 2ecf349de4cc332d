"""tools/rehearse_405b_shared.py on CPU at a tiny width: the 2-D + offload layout (tp 2 x dp 2, 4
gloo ranks) and the single-process oracle load the same safetensors weights and agree on the
losses and on every parameter's update (the same tool runs at 405B width on the GPU,
gpujobs/r6_405b_shared.sh)."""
import json
import os
import subprocess
import sys

import pytest

from _dist import free_port

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOL = os.path.join(ROOT, "tools", "rehearse_405b_shared.py")


@pytest.mark.slow
def test_rehearsal_tool_2d_offload_matches_oracle(tmp_path):
    env = dict(os.environ, OMP_NUM_THREADS="2")
    common = ["--model", "llama-tiny-d128", "--dir", str(tmp_path / "w"), "--layers", "2", "--seq", "64"]
    r = subprocess.run([sys.executable, TOOL, "prep"] + common, capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    r = subprocess.run([sys.executable, TOOL, "run"] + common + ["--tp", "1", "--batch", "2", "--out",
                                                                 str(tmp_path / "o.json")],
                       capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "4",
                        "--master-addr", "127.0.0.1", "--master-port", str(free_port()), TOOL, "run"] + common
                       + ["--tp", "2", "--batch", "1", "--out", str(tmp_path / "t.json")],
                       capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    r = subprocess.run([sys.executable, TOOL, "compare", str(tmp_path / "o.json"), str(tmp_path / "t.json")],
                       capture_output=True, text=True, env=env, timeout=120)
    rec = json.loads(r.stdout.strip().splitlines()[-1])
    assert r.returncode == 0 and rec["match"], rec
    assert rec["worst_loss_rel"] < 1e-3 and rec["worst_update_sumsq_rel"] < 1e-2
    twod = json.load(open(tmp_path / "t.json"))
    assert twod["world"] == 4 and twod["tp"] == 2 and twod["dp"] == 2
