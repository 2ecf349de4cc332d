"""Auxiliary subsystems that PARITY.md listed without a covering test: the cluster monitor
(reference top-cluster.py), LR scaling (F4), the JSONL metric sink (H3/H4),
the launcher environment contract (I3) and the packed data-loader benchmark (E8)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import dtg  # noqa: E402,F401


def _amd_smi_metric(n, power, util=90):
    return json.dumps([
        {"gpu": i,
         "usage": {"gfx_activity": {"value": util, "unit": "%"}},
         "power": {"socket_power": {"value": power, "unit": "W"},
                   "power_limit": {"value": 1400, "unit": "W"}},
         "mem_usage": {"used_vram": {"value": 144 * 1024, "unit": "MB"},
                       "total_vram": {"value": 288 * 1024, "unit": "MB"}}}
        for i in range(n)])


def _amd_smi_process(n, per_gpu):
    return json.dumps([{"gpu": i, "process_list": [{"process_info": {"pid": 100 + j}}
                                                   for j in range(per_gpu)]} for i in range(n)])


def test_cluster_monitor_parses_amd_smi_and_summarizes():
    import top_cluster as tc

    gpus = tc.parse_amd_smi(_amd_smi_metric(8, 1120), _amd_smi_process(8, 1))
    assert len(gpus) == 8
    assert gpus[0]["util"] == 90 and gpus[0]["power"] == 1120 and gpus[0]["nprocs"] == 1
    s = tc.summarize(gpus)
    assert s["power"] == pytest.approx(80.0)
    assert s["mem"] == pytest.approx(50.0)
    assert s["nprocs"] == 8
    # the hang signature: processes present, power near idle
    idle = tc.summarize(tc.parse_amd_smi(_amd_smi_metric(8, 140, util=100), _amd_smi_process(8, 1)))
    assert idle["power"] < 20 and idle["nprocs"] > 0
    # missing / malformed tool output degrades to "no data", not an exception
    assert tc.summarize(tc.parse_amd_smi("", "")) is None
    assert tc.parse_amd_smi(_amd_smi_metric(2, 500), "not json")[1]["nprocs"] == 0


def test_cluster_monitor_dict_layout_and_defaults():
    import top_cluster as tc

    data = json.dumps({"gpu_data": [{"usage": {"gfx_usage": 12}, "power": {"current_socket_power": 700},
                                     "vram": {"vram_used": 1024}}]})
    (g,) = tc.parse_amd_smi(data, "[]")
    assert g["util"] == 12 and g["power"] == 700
    assert g["power_cap"] == 1400.0 and g["mem_total"] == 288 * 1024.0


def test_lr_scaling_rules():
    from dtg.utils.lr_scaling import effective_batch, scale_lr

    assert effective_batch(16, 8, 4) == 512
    assert scale_lr(3e-5, 16, 128, "linear") == pytest.approx(2.4e-4)
    assert scale_lr(3e-5, 16, 64, "sqrt") == pytest.approx(6e-5)
    assert scale_lr(1e-3, 32, 32) == pytest.approx(1e-3)
    with pytest.raises(ValueError):
        scale_lr(1e-3, 1, 2, "cubic")


def test_metric_sink_writes_per_rank_jsonl(tmp_path, monkeypatch):
    from dtg.utils.metrics import MetricSink

    monkeypatch.setenv("DTG_NO_WANDB", "1")
    sink = MetricSink(tmp_path, rank=3)
    assert sink.wandb is None
    sink.log({"loss": 2, "lr": 3e-5, "tag": "x"}, step=1)
    sink.log({"loss": 1.5}, step=2)
    lines = (tmp_path / "metrics-rank3.jsonl").read_text().splitlines()
    recs = [json.loads(l) for l in lines]
    assert recs[0] == {"loss": 2.0, "lr": 3e-5, "tag": "x"} and isinstance(recs[0]["loss"], float)
    assert recs[1]["loss"] == 1.5


@pytest.mark.parametrize("script", ["torchrun_single_node.sh", "launch_ssh_tmux.sh", "mpirun.sh", "job.sbatch"])
def test_launchers_export_env_contract(script):
    import re

    text = open(os.path.join(ROOT, "03-job-launchers", script)).read()
    # dmabuf IPC is the only mode the ROCm driver supports for RCCL / tensor sharing
    assert re.search(r"HSA_ENABLE_IPC_MODE_LEGACY(=|:-)0", text)
    assert re.search(r"OMP_NUM_THREADS(=|:-)1", text)


def test_torchrun_launcher_env_and_command(tmp_path):
    """Runs the single-node launcher with a stub `python` on PATH that records its env/argv."""
    stub = tmp_path / "python"
    stub.write_text("#!/bin/bash\n"
                    "echo \"$TORCHELASTIC_ERROR_FILE|$OMP_NUM_THREADS|$HSA_ENABLE_IPC_MODE_LEGACY\" > \"$STUB_OUT\"\n"
                    "echo \"$@\" >> \"$STUB_OUT\"\n")
    stub.chmod(0o755)
    out = tmp_path / "rec.txt"
    env = {k: v for k, v in os.environ.items()
           if k not in ("TORCHELASTIC_ERROR_FILE", "OMP_NUM_THREADS", "HSA_ENABLE_IPC_MODE_LEGACY")}
    env.update(PATH=f"{tmp_path}:{env.get('PATH', '')}", STUB_OUT=str(out))
    r = subprocess.run(["bash", "torchrun_single_node.sh", "02-distributed-data-parallel", "-e", "x", "-b", "4"],
                       cwd=os.path.join(ROOT, "03-job-launchers"), env=env, capture_output=True, text=True,
                       timeout=60)
    assert r.returncode == 0, r.stderr
    envline, argv = out.read_text().splitlines()
    assert envline == "../error.json|1|0"
    assert "torch.distributed.run" in argv and "--nproc-per-node gpu" in argv
    assert argv.endswith("../02-distributed-data-parallel/train_llm.py -e x -b 4")


def test_dataloader_bench_runs_and_reports(tmp_path):
    env = dict(os.environ, PYTHONPATH=ROOT, WORLD_SIZE="1", RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "bench_dataloader.py"),
                        "--batches", "20", "--seq-length", "1024", "--num-workers", "0", "--json"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=tmp_path)
    assert r.returncode == 0, r.stderr[-2000:]
    rec = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert rec["world"] == 1 and rec["tokens"] == 20 * 1024
    assert rec["tok_per_s_total"] > 0


def test_collectives_bench_gloo_rehearsal():
    """tools/bench_collectives.py harness at world 2 on gloo: every op reports
    nccl-tests style algbw / busbw with the right bus factor."""
    from _dist import free_port

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.join(ROOT, "tools", "bench_collectives.py"), "--backend", "gloo", "--json",
           "--min-mb", "0.25", "--max-mb", "0.5", "--iters", "2", "--warmup", "1"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=dict(os.environ, OMP_NUM_THREADS="1"))
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    recs = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert {x["op"] for x in recs} == {"all_reduce", "all_gather", "reduce_scatter", "all_to_all"}
    assert len(recs) == 8 and all(x["world"] == 2 and x["time_us"] > 0 for x in recs)
    for x in recs:
        factor = 1.0 if x["op"] == "all_reduce" else 0.5  # 2(n-1)/n and (n-1)/n at n = 2
        assert x["busbw_GBps"] == pytest.approx(x["algbw_GBps"] * factor, rel=0.02, abs=0.02)


@pytest.mark.parametrize("mode", ["rank0", "local_rank0", "every_rank"])
def test_wandb_init_kwargs_per_mode(tmp_path, mode):
    """The reference's three wandb layouts (related-topics/wandb-configurations): which ranks log,
    and the id / name / group / dir / save_code / resume of their runs.  4 ranks, 2 per node."""
    from dtg.utils.metrics import wandb_init_kwargs

    got = {r: wandb_init_kwargs(mode, tmp_path, "exp", r, r % 2, resumed=(r == 1), config={"a": 1}) for r in range(4)}
    logging_ranks = [r for r, kw in got.items() if kw is not None]
    assert logging_ranks == {"rank0": [0], "local_rank0": [0, 2], "every_rank": [0, 1, 2, 3]}[mode]
    for r in logging_ranks:
        kw = got[r]
        assert kw["project"] == "distributed-training-guide" and kw["save_code"] is True and kw["config"] == {"a": 1}
        assert kw["resume"] == ("must" if r == 1 else None)
        if mode == "rank0":
            assert (kw["id"], kw["name"], kw["dir"]) == ("exp", "exp", str(tmp_path)) and "group" not in kw
        else:
            assert (kw["id"], kw["name"], kw["group"]) == (f"exp-{r}", f"rank-{r}", "exp")
            assert kw["dir"] == str(tmp_path / f"rank-{r}") and (tmp_path / f"rank-{r}").is_dir()


def test_trainer_wandb_every_rank_with_stub_module(tmp_path):
    """Chapter 02 on 2 gloo ranks with a stub `wandb` module on the path: every rank opens its own
    grouped run with the reference's kwargs and logs its metric records to it."""
    import subprocess
    import sys

    from _dist import free_port

    stub = tmp_path / "stub"
    stub.mkdir()
    (stub / "wandb.py").write_text(
        "import json, os\n"
        "_out = os.environ['WANDB_STUB_OUT']\n"
        "def init(**kw):\n"
        "    global _id\n"
        "    _id = kw['id']\n"
        "    kw = {k: v for k, v in kw.items() if k != 'config'}\n"
        "    json.dump(kw, open(os.path.join(_out, 'init-' + _id + '.json'), 'w'))\n"
        "def log(info, step=None):\n"
        "    open(os.path.join(_out, 'log-' + _id + '.txt'), 'a').write(str(step) + '\\n')\n")
    out = tmp_path / "out"
    out.mkdir()
    env = dict(os.environ, OMP_NUM_THREADS="1", PYTHONPATH=f"{stub}:{os.environ.get('PYTHONPATH', '')}",
               WANDB_STUB_OUT=str(out))
    env.pop("DTG_NO_WANDB", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.join(ROOT, "02-distributed-data-parallel", "train_llm.py"),
           "-e", "wb", "-m", "llama-tiny", "-d", "synthetic", "-b", "2", "-s", "64", "--max-steps", "2",
           "--log-freq", "1", "--save-dir", str(tmp_path / "runs"), "--wandb-mode", "every_rank"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=400, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    for rank in (0, 1):
        kw = json.loads((out / f"init-wb-{rank}.json").read_text())
        assert (kw["group"], kw["name"], kw["save_code"]) == ("wb", f"rank-{rank}", True)
        assert kw["dir"].endswith(f"wb/rank-{rank}")
        assert (out / f"log-wb-{rank}.txt").read_text().split() == ["1", "2"]


def test_num_layers_flag_builds_reduced_depth():
    """--num-layers overrides the bundled config's depth (exact-width reduced-depth runs such
    as chapter 05 at the 405B width, tools/run_405b_gpu.sh); absent, the config's depth."""
    import torch

    from dtg.train import trainer
    from dtg.train.cli import get_parser

    for argv, depth in ((["--num-layers", "3"], 3), ([], None)):
        args = get_parser("01").parse_args(["-e", "x", "-d", "synthetic", "-m", "llama-tiny"] + argv)
        model = trainer._build(args, "01", torch.device("cpu"), 1)[0]
        want = depth if depth is not None else trainer.resolve_config("llama-tiny").num_hidden_layers
        assert len(model.layers) == want


def _ch05_log(path, fwd, bwd, upd):
    lines = []
    for step in range(1, 7):
        rec = {"global_step": step, "time/forward": fwd, "time/backward": bwd, "time/update": upd,
               "time/total": fwd + bwd + upd}
        lines.append(f"[rank=0] INFO:{rec!r}")
    path.write_text("\n".join(lines) + "\n")


def test_extrapolate_405b_from_depth_logs(tmp_path):
    """Per-layer costs = (depth 4 - depth 2) / 2 of the chapter-05 phase timers; the projection
    reports compute-only and the two labelled recipes."""
    _ch05_log(tmp_path / "ch05_405b_d2_no_offload.log", 82.0, 141.0, 29.7)
    _ch05_log(tmp_path / "ch05_405b_d4_no_offload.log", 122.2, 275.0, 43.0)
    _ch05_log(tmp_path / "ch05_405b_d2.log", 82.0, 511.0, 339.0)
    _ch05_log(tmp_path / "ch05_405b_d4.log", 122.2, 835.0, 602.0)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "extrapolate_405b.py"), str(tmp_path)],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    res = json.loads(r.stdout)
    m = res["measured"]
    assert abs(m["layer_fwd_ms"] - 20.1) < 0.01 and abs(m["layer_bwd_ms"] - 67.0) < 0.01
    assert abs(m["compute_only_step_s"] - (126 * 87.1 + 49.2) / 1e3) < 0.02
    assert res["A_full_shard_offload"]["tok_s_gpu"] < res["B_hybrid_xgmi_optimizer_offload"]["tok_s_gpu"]
    assert res["reference_tok_s_gpu"] == 136.5


def test_ce_overlap_pairs_chunks_in_order(tmp_path):
    """tools/ce_overlap.py on a synthetic trace of the pipelined vocab-parallel loss head:
    issue(0) issue(1) finish(0) issue(2) finish(1) finish(2) -> 2 of 3 chunks pipelined."""
    ev, t = [], 0

    def k(name, dur=10):
        nonlocal t
        ev.append((t, t + dur, name))
        t += dur

    for j in range(2):
        k("Cijk_gemm_logits")
        k("dtg::ce_stats_kernel()")
        k("dtg::xgmi::barrier_kernel()", 1)
    k("dtg::ce_grad_kernel()")
    k("Cijk_gemm_logits")
    k("dtg::ce_stats_kernel()")
    k("dtg::ce_grad_kernel()")
    k("dtg::ce_grad_kernel()")
    d = tmp_path / "trace"
    d.mkdir()
    with open(d / "123_run_kernel_trace.csv", "w") as fp:
        fp.write("Kernel_Name,Start_Timestamp,End_Timestamp\n")
        for s, e, n in ev:
            fp.write(f"\"{n}\",{s},{e}\n")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "ce_overlap.py"), str(d)],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    assert "3 ce_stats, 3 ce_grad" in r.stdout and "2 / 3" in r.stdout, r.stdout


def test_fake_world_runs_one_rank_of_a_larger_job(tmp_path):
    """DTG_FAKE_WORLD=W: chapter 05 (FSDP + AC + offload) runs as rank 0 of a W-rank job with a
    fake process group for the others; the shard is 1/W of the model (memory / per-rank compute
    rehearsal; numerics not meaningful)."""
    env = dict(os.environ, DTG_FAKE_WORLD="8", OMP_NUM_THREADS="1")
    cmd = [sys.executable, "train_llm.py", "-e", "fw", "-m", "llama-tiny", "-b", "1", "-s", "64", "-d", "synthetic",
           "--save-dir", str(tmp_path), "--ckpt-freq", "1000", "--max-steps", "2", "--log-freq", "1",
           "--num-workers", "0"]
    r = subprocess.run(cmd, cwd=os.path.join(ROOT, "05-training-llama-405b"), env=env, capture_output=True,
                       text=True, timeout=300)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-3000:]
    assert "'global_step': 2" in out, out[-3000:]


def test_fake_world_2d_rehearsal_stays_finite(tmp_path):
    """DTG_FAKE_WORLD=8 with chapter 07's 2-D mesh (tp 2 x dp 4): the fake group's collectives
    leave their outputs untouched, so utils/comm.py fills them with this rank's data; without
    that the sequence-parallel gathers read uninitialised memory and the loss turns NaN after
    one step.  Every logged loss is finite."""
    import math
    import re

    env = dict(os.environ, DTG_FAKE_WORLD="8", OMP_NUM_THREADS="1")
    cmd = [sys.executable, "train_llm.py", "-e", "fw2d", "-m", "llama-tiny-d128", "-b", "2", "-s", "64", "-d",
           "synthetic", "--save-dir", str(tmp_path), "--ckpt-freq", "1000", "--max-steps", "3", "--log-freq", "1",
           "--num-workers", "0", "--tp", "2", "--cpu-offload", "on", "--offload-params", "off"]
    r = subprocess.run(cmd, cwd=os.path.join(ROOT, "07-2d-parallel"), env=env, capture_output=True, text=True,
                       timeout=300)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-3000:]
    losses = [float(x) for x in re.findall(r"'running_loss': ([0-9.eEna+-]+)", out)]
    assert len(losses) >= 3 and all(math.isfinite(x) for x in losses), losses


def test_fake_world_vocab_parallel_embedding_has_no_zero_rows(monkeypatch):
    """Under DTG_FAKE_WORLD the vocab-parallel embedding's sum over TP ranks never arrives, so a
    token outside this rank's shard would get an all-zero row.  The first token of a sequence then
    stays zero through every layer, and the RMSNorm backward overflows bf16
    (profiles/r5/fake_nan/).  In the rehearsal every token takes a row of this shard; outside it,
    the masking is unchanged."""
    import torch

    from dtg.models import llama
    from dtg.utils import comm

    w = torch.randn(16, 8)
    ids = torch.arange(64)  # vocab 64 over 4 ranks; this rank holds rows 16..31
    monkeypatch.setattr(comm, "_FAKE", False)
    real = llama._VocabParallelEmbedding.apply(ids, w, 16)
    assert int((real.abs().sum(1) == 0).sum()) == 48
    monkeypatch.setattr(comm, "_FAKE", True)
    fake = llama._VocabParallelEmbedding.apply(ids, w, 16)
    assert bool((fake.abs().sum(1) > 0).all())
    assert torch.equal(fake[16:32], real[16:32])
