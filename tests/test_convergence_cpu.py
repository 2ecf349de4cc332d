"""The training stack LEARNS: chapter 01's trainer on `synthetic:pattern` (arithmetic
progressions mod V, data/synthetic.py SyntheticPattern) drives the loss from ln V far down.
Uniform random tokens -- the benchmark data -- cannot show this: their loss stays at ln V for a
correct and a broken stack alike.  The GPU twin (tests/test_convergence_gpu.py) runs the same
check through the HIP kernels."""
import json
import math
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_pattern(tmp_path, extra=(), steps=160, timeout=600, chapter="01-single-gpu", nproc=0):
    """Train on synthetic:pattern; nproc > 0 launches `nproc` gloo ranks through torchrun."""
    launch = [sys.executable]
    if nproc:
        from _dist import free_port

        launch += ["-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(nproc),
                   "--master-addr", "127.0.0.1", "--master-port", str(free_port())]
    cmd = launch + ["train_llm.py", "-e", "cv", "-m", "llama-tiny", "-d", "synthetic:pattern", "-b", "16",
           "-s", "64", "--lr", "3e-3", "--num-workers", "0", "--log-freq", "20", "--ckpt-freq", "100000",
           "--max-steps", str(steps), "--save-dir", str(tmp_path), *extra]
    env = dict(os.environ, DTG_NO_WANDB="1")
    if nproc:
        env["OMP_NUM_THREADS"] = "1"  # the ranks share the 8 CPUs
    r = subprocess.run(cmd, cwd=os.path.join(ROOT, chapter), capture_output=True, text=True, timeout=timeout, env=env)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    recs = [json.loads(x) for x in (tmp_path / "cv" / "metrics-rank0.jsonl").read_text().splitlines()]
    return [x["running_loss"] for x in recs if x["global_step"] > 0]


def test_pattern_data_is_learned(tmp_path):
    losses = run_pattern(tmp_path)
    assert math.log(512) * 0.6 < losses[0]  # starts near ln V (llama-tiny: V = 512; window mean of steps 1-20)
    assert losses[-1] < 1.5 and losses[-1] < losses[0] / 3, losses


def test_pattern_data_is_learned_2d_tp2_dp2(tmp_path):
    """Chapter 07's FSDP x TP (tp 2 x dp 2, four gloo ranks, real collectives) learns too."""
    losses = run_pattern(tmp_path, ("-b", "8", "--tp", "2"), steps=120, chapter="07-2d-parallel", nproc=4)
    assert math.log(512) * 0.6 < losses[0]
    assert losses[-1] < losses[0] / 2.5, losses


def test_pattern_data_is_learned_fsdp_offload(tmp_path):
    """Chapter 05's FSDP with CPU offload (host AdamW) on two gloo ranks learns too."""
    losses = run_pattern(tmp_path, ("-b", "8", "--cpu-offload", "on"), steps=120, chapter="05-training-llama-405b", nproc=2)
    assert math.log(512) * 0.6 < losses[0]
    assert losses[-1] < losses[0] / 2.5, losses


@pytest.fixture(scope="module")
def single_b8(tmp_path_factory):
    """One process, batch 8, chapter 02: the curve the split runs must follow."""
    return run_pattern(tmp_path_factory.mktemp("single"), ("-b", "8"), steps=100, chapter="02-distributed-data-parallel")


@pytest.mark.parametrize("split", ["--cp", "--sp", "--pp"])
def test_pattern_data_is_learned_split_like_one_process(tmp_path, single_b8, split):
    """Context parallel (zig-zag shards), Ulysses (seq <-> heads all-to-all) and 1F1B pipeline
    parallel (two decoder-layer stages, 4 micro-batches) each split the work of one batch over two
    ranks: they learn like one process with the same batch (the splits change no value beyond
    rounding: tests/test_cp_cpu.py, tests/test_ulysses_cpu.py, tests/test_pipeline_cpu.py)."""
    losses = run_pattern(tmp_path, ("-b", "8", split, "2"), steps=100, chapter="02-distributed-data-parallel", nproc=2)
    assert losses[-1] < losses[0] / 1.6, losses
    assert abs(losses[-1] - single_b8[-1]) < 0.1 * single_b8[-1], (losses, single_b8)
