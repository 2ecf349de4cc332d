"""Transport selection by measurement (`--tp-comm auto` / `--dp-comm auto`, parallel/transport.py)
on gloo ranks with stubbed timings: the slowest rank's time decides, every rank picks the same
transport, a candidate that fails on any rank is never picked, RCCL wins ties and near-ties (margin)."""
import math

import pytest

from _dist import run_distributed


def _stub_pick(rank, world, times, fail_on):
    from dtg.parallel import transport

    def time_fn(c):
        if (c.name, rank) in fail_on:
            raise RuntimeError(f"{c.name} broke on rank {rank}")
        return times[c.name][rank]

    return transport.select("tp", None, "cpu", 16 << 20, time_fn=time_fn)


def test_select_uses_the_slowest_rank_and_agrees():
    # xgmi is fastest on rank 0 but slowest on rank 1; xgmi-dma's worst rank is the best worst
    times = {"rccl": [3e-4, 3e-4], "xgmi": [1e-4, 5e-4], "xgmi-dma": [2e-4, 2.5e-4]}
    res = run_distributed(_stub_pick, 2, times, set())
    (c0, t0), (c1, t1) = res
    assert c0 == c1 == "xgmi-dma"
    assert t0 == t1
    assert t0["xgmi"]["us"] == pytest.approx(500.0) and t0["rccl"]["us"] == pytest.approx(300.0)
    assert t0["xgmi-dma"]["msg_mib"] == 16.0


def test_select_excludes_a_candidate_that_fails_anywhere():
    times = {"rccl": [3e-4, 3e-4], "xgmi": [1e-4, 1e-4], "xgmi-dma": [2e-4, 2e-4]}
    res = run_distributed(_stub_pick, 2, times, {("xgmi", 1)})
    (c0, t0), (c1, t1) = res
    assert c0 == c1 == "xgmi-dma"
    assert t0["xgmi"]["us"] is None and t0["xgmi"]["error"] == "failed on another rank"
    assert "broke on rank 1" in t1["xgmi"]["error"]


def test_pick_prefers_rccl_on_ties_and_without_data():
    from dtg.parallel.transport import pick

    assert pick({"rccl": {"us": 10.0}, "xgmi-dma": {"us": 10.0}}) == "rccl"
    assert pick({"rccl": {"us": None}, "xgmi-dma": {"us": None}}) == "rccl"
    assert pick({"rccl": {"us": 12.0}, "xgmi-dma": {"us": 9.0}}) == "xgmi-dma"
    # an alternative within the margin of RCCL (10 % by default) does not displace it
    assert pick({"rccl": {"us": 10.0}, "xgmi-dma": {"us": 9.5}}) == "rccl"
    assert pick({"rccl": {"us": 10.0}, "xgmi-dma": {"us": 9.5}}, margin=0.0) == "xgmi-dma"
    assert pick({"rccl": {"us": None}, "xgmi-dma": {"us": 9.5}}) == "xgmi-dma"


def _cpu_auto(rank, world):
    from dtg.parallel import transport

    return transport.resolve("auto", "dp", None, "cpu", 64 << 20), transport.resolve("xgmi", "tp", None, "cpu", 1)


def test_resolve_on_cpu_is_the_process_group():
    (auto, explicit), _ = run_distributed(_cpu_auto, 2)
    assert auto[0] == "rccl" and "CPU" in auto[1]["rccl"]["note"]
    assert explicit == ("xgmi", None)


def test_trainer_and_bench_default_to_rccl():
    """The trainer's chapters and the bench default to RCCL; auto (the child-job calibration) is
    opt-in until a multi-GPU run has validated the direct-peer paths."""
    import bench
    from dtg.train.cli import get_parser

    for ch in ("06", "07"):
        a = get_parser(ch).parse_args(["-e", "x", "-d", "synthetic", "-m", "llama-tiny"])
        assert a.tp_comm == "rccl"
    for ch in ("02", "04", "05", "07"):
        a = get_parser(ch).parse_args(["-e", "x", "-d", "synthetic", "-m", "llama-tiny"])
        assert a.dp_comm == "rccl"
    b = bench.parse([])
    assert b.tp_comm == "rccl" and b.dp_comm == "rccl"
    assert math.isfinite(b.deadline_s) and b.diag_budget_s < b.deadline_s


def _isolated(rank, world, stub, timeout):
    import json
    import os

    from dtg.parallel import transport

    os.environ["DTG_TRANSPORT_CHILD_CMD"] = json.dumps(stub)
    logged = []
    out = transport.resolve_isolated("auto", "tp", "cpu", 8 << 20, mesh=(world, 1), log=logged.append,
                                     child_timeout=timeout)
    return out, logged


def test_isolated_calibration_child_crash_falls_back_to_rccl():
    import sys

    res = run_distributed(_isolated, 2, [sys.executable, "-c", "import sys; sys.exit(3)"], 60)
    for (choice, table), logged in res:
        assert choice == "rccl"
        assert "exited 3" in table["child"]["error"]
    assert "-> rccl" in res[0][1][0] and "exited 3" in res[0][1][0]


def test_isolated_calibration_child_timeout_falls_back_to_rccl():
    import sys

    res = run_distributed(_isolated, 2, [sys.executable, "-c", "import time; time.sleep(30)"], 2)
    assert all(c == "rccl" and "timed out" in t["child"]["error"] for (c, t), _ in res)


def test_isolated_calibration_every_rank_takes_the_childs_pick():
    import json
    import sys

    rec = {"choice": "xgmi-dma", "table": {"rccl": {"us": 30.0}, "xgmi": {"us": 25.0}, "xgmi-dma": {"us": 20.0}}}
    res = run_distributed(_isolated, 2, [sys.executable, "-c", f"print({json.dumps(json.dumps(rec))})"], 60)
    assert [c for (c, _), _ in res] == ["xgmi-dma", "xgmi-dma"]
    bad = dict(rec, choice="nvlink")
    res = run_distributed(_isolated, 2, [sys.executable, "-c", f"print({json.dumps(json.dumps(bad))})"], 60)
    assert all(c == "rccl" and "picked 'nvlink'" in t["child"]["error"] for (c, t), _ in res)


def test_real_calibration_child_runs_on_cpu():
    """The real child script under torchrun (2 gloo ranks on the CPU: the process group's own
    collectives, recorded with the CPU note)."""
    from dtg.parallel import transport

    rec = transport.run_child(2, {"kind": "dp", "msg_bytes": 1 << 20, "mesh": [1, 0], "timeout_s": None}, 240)
    assert rec.get("choice") == "rccl", rec
    assert "CPU" in rec["table"]["rccl"]["note"]
