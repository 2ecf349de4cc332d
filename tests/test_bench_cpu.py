"""bench.py's driver contract on CPU ranks: one JSON line from rank 0 with the BASELINE metric,
whole-job tokens/s, n_gpus / steps / warmup echoed, weak-scaling global batch, for N=1 and for
torchrun N=2 (gloo)."""
import json
import os
import subprocess
import sys

import pytest

from _dist import free_port

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--steps", "2", "--warmup", "1", "--model", "llama-tiny", "--batch-size", "2", "--seq-len", "64",
        "--tunableop", "off"]


def _json_lines(out):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{")]


def _check(rec, n):
    assert rec["metric"].startswith("tokens/sec/GPU")
    assert rec["n_gpus"] == n and rec["steps"] == 2 and rec["warmup"] == 1
    assert rec["config"]["global_batch"] == 2 * n and rec["config"]["seq_len"] == 64
    assert rec["scaling"] == "weak" and rec["higher_is_better"] is True and rec["dtype"] == "bf16"
    assert rec["value"] > 0 and abs(rec["value"] - 2 * n * 64 * 2 / (rec["ms_per_step"] * 2 / 1000)) < 0.02 * rec["value"]


@pytest.mark.slow
def test_bench_single_process():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1"] + ARGS,
                       capture_output=True, text=True, timeout=300, env=dict(os.environ, OMP_NUM_THREADS="2"))
    assert r.returncode == 0, r.stderr[-2000:]
    recs = _json_lines(r.stdout)
    assert len(recs) == 1
    _check(recs[0], 1)


@pytest.mark.slow
def test_bench_torchrun_two_ranks():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2"] + ARGS
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=dict(os.environ, OMP_NUM_THREADS="2"))
    assert r.returncode == 0, r.stderr[-3000:]
    recs = _json_lines(r.stdout)
    assert len(recs) == 1, r.stdout  # rank 0 only
    _check(recs[0], 2)
    assert recs[0]["config"]["parallelism"] == "dp2-zero"
