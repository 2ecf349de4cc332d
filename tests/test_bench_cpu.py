"""bench.py's driver contract on CPU ranks: one JSON line from rank 0 with the BASELINE metric,
whole-job tokens/s, n_gpus / steps / warmup echoed, weak-scaling global batch, for N=1 and for
torchrun N=2 (gloo)."""
import json
import math
import os
import subprocess
import sys

import pytest

from _dist import free_port

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--steps", "2", "--warmup", "1", "--model", "llama-tiny", "--batch-size", "2", "--seq-len", "64",
        "--tunableop", "off", "--fsdp-mem-model", "llama-tiny", "--fsdp-mem-batch", "2", "--fsdp-mem-seq", "64",
        "--fsdp-mem-steps", "1", "--numel-to-wrap", "10000", "--coll-sweep-mb", "1,2",
        "--bucket-sweep-mb", "1,4", "--sweep-steps", "1", "--ref-steps", "2"]


def _json_lines(out):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{")]


def _check(rec, n):
    assert rec["metric"].startswith("tokens/sec/GPU")
    assert rec["n_gpus"] == n and rec["steps"] == 2 and rec["warmup"] == 1
    assert rec["config"]["global_batch"] == 2 * n and rec["config"]["seq_len"] == 64
    assert rec["scaling"] == "weak" and rec["higher_is_better"] is True and rec["dtype"] == "bf16"
    assert rec["value"] > 0 and abs(rec["value"] - 2 * n * 64 * 2 / (rec["ms_per_step"] * 2 / 1000)) < 0.02 * rec["value"]
    assert rec["world_size_seen_by_pg"] == n and len(rec["rank_devices"]) == n
    assert rec["rank_ms_per_step"]["max"] >= rec["rank_ms_per_step"]["min"] > 0
    assert rec["fsdp_mem"]["peak_gb_max_rank"] >= rec["fsdp_mem"]["valley_gb_max_rank"] >= 0
    # fresh uniform ids every step: the loss is a tripwire around ln(V) (llama-tiny: V = 512)
    lo, hi = rec["loss_band"]
    assert lo < rec["final_loss"] < hi and abs(rec["final_loss"] - math.log(512)) < 0.5
    # reference-mode throughput (synchronised phase timers) next to the async headline
    assert rec["reference_timer_steps"] == 2 and rec["tok_s_reference_timers"] > 0
    assert set(rec["reference_timer_ms"]) == {"data", "forward", "backward", "update"}
    if n > 1:  # the collective sweep after the timed region (gloo: all-gather + all-reduce)
        ops = {(c["op"], c["mib"]) for c in rec["collectives"]}
        assert {("all_gather", 1), ("all_reduce", 2)} <= ops
        assert all(c["busbw_gbs"] > 0 for c in rec["collectives"])
        assert rec["replicas_consistent"] is True
        if rec["config"]["parallelism"].startswith(f"dp{n}-"):
            assert [r["bucket_mb"] for r in rec["bucket_sweep"]] == [1, 4]
            assert all(r["ms_per_step"] > 0 for r in rec["bucket_sweep"])
        assert "rccl" not in rec  # gloo: no RCCL communicator to diagnose
    else:
        assert "collectives" not in rec and "bucket_sweep" not in rec and "replicas_consistent" not in rec


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


@pytest.mark.slow
def test_bench_self_launches_n_ranks():
    """`python bench.py --gpus 2` with no launcher starts the 2 ranks itself (the driver's
    N=1 command form must not silently measure one rank at N>1)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["OMP_NUM_THREADS"] = "2"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"] + ARGS,
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    recs = _json_lines(r.stdout)
    assert len(recs) == 1, r.stdout
    _check(recs[0], 2)
    assert recs[0]["backend"] == "gloo"


def test_bench_rejects_world_mismatch():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"] + ARGS,
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode != 0 and "WORLD_SIZE=1" in (r.stderr + r.stdout)


@pytest.mark.slow
def test_bench_tensor_parallel_two_ranks():
    """BASELINE config 06 shape: `--tp 2` on 2 ranks is one TP group (dp = 1), so a step is
    1 x B x S tokens (the reference's TP formula) and both ranks train the same batch."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--tp", "2"] + ARGS
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=dict(os.environ, OMP_NUM_THREADS="2"))
    assert r.returncode == 0, r.stderr[-3000:]
    recs = _json_lines(r.stdout)
    assert len(recs) == 1, r.stdout
    rec = recs[0]
    assert rec["n_gpus"] == 2 and rec["config"]["global_batch"] == 2
    assert rec["config"]["parallelism"] == "dp1-single-tp2-gloo"  # TP collectives on the PG backend
    assert abs(rec["value"] - 2 * 64 * 2 / (rec["ms_per_step"] * 2 / 1000)) < 0.02 * rec["value"]


@pytest.mark.slow
def test_bench_fake_world_rehearsal_is_labelled():
    """DTG_FAKE_WORLD=8: rank 0 of the 8-rank job alone (fake process group for the others).
    The line is labelled a rehearsal, carries no collective sweep, and its tokens/s counts
    8 ranks' worth of batches."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(OMP_NUM_THREADS="2", DTG_FAKE_WORLD="8")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8"] + ARGS,
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    recs = _json_lines(r.stdout)
    assert len(recs) == 1, r.stdout
    rec = recs[0]
    assert rec["metric"].startswith("REHEARSAL") and "fake process group" in rec["rehearsal"]
    assert rec["backend"] == "fake" and rec["world_size_seen_by_pg"] == 8 and rec["rank_devices"] == [0]
    assert rec["config"]["global_batch"] == 16 and rec["config"]["parallelism"] == "dp8-zero"
    assert "collectives" not in rec
    assert abs(rec["value"] - 8 * 2 * 64 * 2 / (rec["ms_per_step"] * 2 / 1000)) < 0.02 * rec["value"]


RCCL_LOG = """\
box:1234:1234 [0] NCCL INFO RCCL version : 2.26.6-HEAD:abcdef
box:1234:1234 [0] NCCL INFO comm 0x55d0 rank 0 nRanks 8 nNodes 1 localRanks 8 localRank 0 MNNVL 0
box:1234:1234 [0] NCCL INFO Channel 00/16 :    0   1   2   3   4   5   6   7
box:1234:1234 [0] NCCL INFO Channel 15/16 :    0   7   6   5   4   3   2   1
box:1234:1234 [0] NCCL INFO 16 coll channels, 16 collnet channels, 0 nvls channels, 32 p2p channels, 4 p2p channels per peer
box:1234:1234 [0] NCCL INFO Channel 00/0 : 0[0] -> 1[1] via P2P/IPC
box:1234:1234 [0] NCCL INFO Channel 01/0 : 0[0] -> 7[7] via P2P/IPC
box:1234:1234 [0] NCCL INFO Channel 02/0 : 0[0] -> 1[1] [send] via SHM/direct/direct
box:1234:1234 [0] NCCL INFO ncclCommInitRankConfig comm 0x55d0 rank 0 nranks 8 cudaDev 0 busId 5000 - Init COMPLETE
"""


def test_rccl_log_parse_and_preset():
    """What the N > 1 bench line reports about RCCL: version, communicator shape, channels and
    the transport of every connection, parsed from its INFO log; the preset never overrides an
    exported variable."""
    from dtg.utils import rccl

    rec = rccl.parse_log(RCCL_LOG)
    assert rec["version"].startswith("2.26.6")
    assert rec["communicators"] == [{"rank": 0, "nranks": 8, "nnodes": 1, "local_ranks": 8}]
    assert rec["channels_max"] == 16 and rec["coll_channels"] == [16] and rec["p2p_channels_per_peer"] == [4]
    assert rec["transports"] == {"P2P/IPC": 2, "SHM/direct/direct": 1}
    env = {"TORCH_NCCL_HIGH_PRIORITY": "0"}
    applied = rccl.apply_preset("node", env)
    assert env["TORCH_NCCL_HIGH_PRIORITY"] == "0" and "TORCH_NCCL_HIGH_PRIORITY" not in applied
    assert applied["HSA_NO_SCRATCH_RECLAIM"] == "1" and rccl.apply_preset("none", env) == {}


@pytest.mark.slow
def test_bench_child_past_its_budget_still_reports():
    """the xGMI child job (stubbed: sleeps far past its timeout) is killed at
    --xgmi-child-timeout; the line still comes out, rc 0, with the child named in
    diagnostic_errors and every phase's wall time recorded."""
    import time

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--diag-stub", "child-sleep:1000", "--xgmi-child-timeout", "15", "--deadline-s", "200"] + ARGS
    t0 = time.time()
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=dict(os.environ, OMP_NUM_THREADS="2"))
    took = time.time() - t0
    assert r.returncode == 0, r.stderr[-3000:]
    recs = _json_lines(r.stdout)
    assert len(recs) == 1, r.stdout
    rec = recs[0]
    _check(rec, 2)
    assert "timed out" in rec["diagnostic_errors"]["xgmi_child"]
    assert rec["xgmi_diag"]["error"].startswith("xgmi diagnostic child timed out")
    assert {"throughput", "collectives", "bucket_sweep", "fsdp_mem", "xgmi_child"} <= set(rec["phase_s"])
    assert 14 <= rec["phase_s"]["xgmi_child"] < 40
    assert rec["wall_s"] > 0 and took < rec["wall_s"] + 60


@pytest.mark.slow
def test_bench_hung_diagnostic_hits_the_deadline():
    """A diagnostic that never returns: at --deadline-s the watchdog prints the headline line
    (with what the diagnostics added so far) and every rank exits 0."""
    import time

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--diag-stub", "hang", "--deadline-s", "40"] + ARGS
    t0 = time.time()
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=dict(os.environ, OMP_NUM_THREADS="2"))
    took = time.time() - t0
    assert r.returncode == 0, r.stderr[-3000:]
    recs = _json_lines(r.stdout)
    assert len(recs) == 1, r.stdout
    rec = recs[0]
    assert rec["value"] > 0 and rec["n_gpus"] == 2
    assert "deadline" in rec["diagnostic_errors"]["stub_hang"]
    assert "collectives" in rec and "bucket_sweep" in rec  # the phases before the hang made it in
    assert 40 <= rec["wall_s"] < 50 and took < 40 + 30


@pytest.mark.slow
def test_bench_diagnostic_budget_skips_phases():
    """With the diagnostic budget already spent, no diagnostic phase starts; each is named."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--diag-budget-s", "0"] + ARGS
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=dict(os.environ, OMP_NUM_THREADS="2"))
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _json_lines(r.stdout)[0]
    assert rec["value"] > 0
    for name in ("collectives", "bucket_sweep", "fsdp_mem"):
        assert "budget" in rec["diagnostic_errors"][name]
    assert "collectives" not in rec and "fsdp_mem" not in rec


def test_bucket_sweep_stops_between_runs_once_the_budget_is_spent():
    """The bucket sweep rebuilds the whole job per size, so it checks the diagnostic budget
    before every run, not only when the phase starts (a 2-rank 8B rehearsal's sweep ran 264 s
    past a phase start at 107 s, profiles/r5/bench2/)."""
    import argparse
    import sys as _sys

    import torch

    _sys.path.insert(0, ROOT)
    import bench

    args = argparse.Namespace(bucket_sweep_mb="1,4", batch_size=2, seq_len=32, dp_comm="rccl", parallel="zero",
                              sweep_other_dp_comm=0, xgmi_child=0, bucket_mb=4, diag_budget_s=-1.0, sweep_steps=1)
    out = bench.bucket_sweep(args, torch, None, torch.device("cpu"), 1, 0, False)
    assert [r.get("skipped") for r in out] == ["diagnostic budget spent"] * 2
