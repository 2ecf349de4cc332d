"""Collective transports chosen by measurement at run time (`--tp-comm auto`, `--dp-comm auto`).

One node of MI355X has three ways to move a tensor-parallel or data-parallel message between
its GPUs: RCCL's ring/tree kernels, this repo's direct-peer pull kernels (`parallel/xgmi.py`,
every GPU reads its 7 peers at once over the point-to-point xGMI links) and the same pulls on
the copy engines (one hipMemcpyAsync stream per peer, no CU time; for data parallel the ZeRO
buffers themselves are shared, `parallel/xgmi_dp.py`).  Which is fastest depends on the message
size, the number of ranks, the RCCL version and its channel count -- so it is measured on the
job's own group at the job's own message sizes, at startup, instead of being a hard-coded default:

    choice, table = select("tp", group, device, msg_bytes=..)      # rccl | xgmi | xgmi-dma
    choice, table = select("dp", group, device, msg_bytes=bucket)  # rccl | xgmi-dma

Each candidate runs its collectives `warmup` + `iters` times; the time of the SLOWEST rank is the
candidate's time (MAX all-reduce), so every rank picks the same winner.  A candidate is also
checked against RCCL's result on integer-valued data (sums exact in any order): one that raises
or disagrees is recorded with its error and never picked.  RCCL comes first and wins ties; an
alternative must be at least 10 % faster than RCCL to be picked (`MARGIN`).
The table ({name: {"us": .., "error": ..}}) is logged by the trainer and recorded by the bench
(`tp_comm_calibration` / `dp_comm_calibration`).

Reference: the reference has one transport, NCCL under DTensor / FSDP
(/root/reference/06-tensor-parallel/train_llm.py:84-128, 04-fully-sharded-data-parallel/
train_llm.py:87-95); the choice exists here because xGMI is point-to-point.
"""
from __future__ import annotations

import math
import os
import time
from typing import Callable, Dict, List, Optional

import torch
import torch.distributed as dist

CANDIDATES = {"tp": ("rccl", "xgmi", "xgmi-dma"), "dp": ("rccl", "xgmi-dma")}


class Candidate:
    """One transport under test: `run()` issues one iteration of the job's collectives on the
    current stream; `verify()` -> bool checks its last result; `close()` releases it."""

    def __init__(self, name: str, run: Callable[[], None], verify: Optional[Callable[[], bool]] = None,
                 close: Optional[Callable[[], None]] = None):
        self.name, self.run, self.verify, self.close = name, run, verify, close


def _device_sync(device):
    if device is not None and torch.device(device).type == "cuda":
        torch.cuda.synchronize(device)


def _all_ok(ok: bool, group, dev) -> bool:
    """Every rank's flag, AND-reduced (a collective every rank issues whatever happened locally)."""
    t = torch.tensor([1.0 if ok else 0.0], dtype=torch.float64,
                     device=dev if (dev.type == "cuda" and dist.get_backend(group) == "nccl") else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return bool(t.item() > 0.5)


def time_candidate(c: Candidate, group, device, warmup: int = 2, iters: int = 5) -> float:
    """Seconds per iteration on this rank (group-synchronised start, device-synchronised end).
    The start is an AND-reduce of "my warmup worked", issued by every rank even when its warmup
    raised, so a rank-local failure cannot leave its peers waiting in a collective."""
    dev = torch.device(device)
    err = None
    try:
        for _ in range(warmup):
            c.run()
        _device_sync(dev)
    except Exception as e:  # noqa: BLE001 - re-raised after the group agreed
        err = e
    if not _all_ok(err is None, group, dev):
        raise err if err is not None else RuntimeError("warmup failed on another rank")
    t0 = time.perf_counter()
    for _ in range(iters):
        c.run()
    _device_sync(dev)
    return (time.perf_counter() - t0) / iters


def measure(builders: Dict[str, Callable[[], Candidate]], group, device, warmup: int = 2, iters: int = 5,
            time_fn: Optional[Callable[[Candidate], float]] = None) -> Dict[str, dict]:
    """{name: {"us": slowest-rank microseconds or None, "error": str?}} in `builders` order.
    `time_fn(candidate) -> seconds` replaces the timing (tests stub it).

    Every rank issues the same collectives whatever fails locally: after build() an AND-reduce
    decides whether anyone times the candidate (a rank whose build raised still joins it), the
    timing starts with another AND-reduce (time_candidate), and a MAX-reduce of the time ends it.
    (A build() that raises BEFORE its own internal exchange, on some ranks only, is the one case
    this cannot cover -- which is why the trainer calibrates in a child job, `resolve_isolated`.)"""
    table: Dict[str, dict] = {}
    dev = torch.device(device) if device is not None else torch.device("cpu")
    for name, build in builders.items():
        err = None
        secs = math.inf
        cand = None
        try:
            cand = build()
        except Exception as e:  # noqa: BLE001 - recorded in the table, the candidate is not picked
            err = repr(e)[:300]
        built = _all_ok(err is None, group, dev)
        if built:
            try:
                secs = time_fn(cand) if time_fn is not None else time_candidate(cand, group, dev, warmup, iters)
                if cand.verify is not None and not cand.verify():
                    err, secs = "result differs from RCCL's", math.inf
            except Exception as e:  # noqa: BLE001
                err, secs = repr(e)[:300], math.inf
        if cand is not None and cand.close is not None:
            try:
                cand.close()
            except Exception as e:  # noqa: BLE001
                err = err or f"close: {e!r}"[:300]
                secs = math.inf
        # the slowest rank bounds the job; a failure anywhere (inf) rules the candidate out everywhere
        t = torch.tensor([secs if math.isfinite(secs) else 1e30], dtype=torch.float64,
                         device=dev if (dev.type == "cuda" and dist.get_backend(group) == "nccl") else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
        worst = float(t.item())
        row = {"us": round(worst * 1e6, 1) if worst < 1e29 else None}
        if err is not None:
            row["error"] = err
        elif worst >= 1e29:
            row["error"] = "failed on another rank"
        table[name] = row
    return table


# An alternative to RCCL must be this much faster to be picked (DTG_TRANSPORT_MARGIN).  RCCL is the
# transport with cross-device mileage; the direct-peer paths are verified against it at startup
# but have run only with every rank on one GPU so far, so a near-tie stays with RCCL.
MARGIN = float(os.environ.get("DTG_TRANSPORT_MARGIN", "0.10"))


def pick(table: Dict[str, dict], default: str = "rccl", margin: float = None) -> str:
    """Fastest candidate with a time; ties go to the earlier one (RCCL first), and a candidate
    other than `default` must beat the default's time by `margin` (a fraction)."""
    margin = MARGIN if margin is None else margin
    best, best_us = default, math.inf
    for name, row in table.items():
        us = row.get("us")
        if us is not None and us < best_us:
            best, best_us = name, us
    d_us = table.get(default, {}).get("us")
    if best != default and d_us is not None and best_us > d_us * (1.0 - margin):
        return default
    return best


# ------------------------------------------------------------------------------------------
# candidate builders
# ------------------------------------------------------------------------------------------
def _pg_all_gather(out, inp, group):
    dist.all_gather_into_tensor(out, inp, group=group)


def _pg_reduce_scatter(out, inp, group):
    """The process group's reduce-scatter (gloo, used by the one-GPU rehearsals, has none:
    all-reduce + own slice, as utils.comm does)."""
    if dist.get_backend(group) == "gloo":
        y = inp.clone()
        dist.all_reduce(y, group=group)
        m = out.numel()
        r = dist.get_rank(group)
        out.copy_(y[r * m:(r + 1) * m])
        return
    dist.reduce_scatter_tensor(out, inp, group=group)


def _int_data(n: int, device, seed: int) -> torch.Tensor:
    """Integer-valued bf16 in [-8, 8]: sums of up to 8 ranks are exact in bf16 in any order."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    return torch.randint(-8, 9, (n,), generator=g).to(device=device, dtype=torch.bfloat16)


def _sizes(msg_bytes: int, world: int):
    n = max(16 * world, (int(msg_bytes) // 2) // (16 * world) * (16 * world))  # bf16 elements, 16-aligned shards
    return n, n // world


def tp_builders(group, device, msg_bytes: int, timeout_s: float = None, candidates=CANDIDATES["tp"]):
    """TP/SP traffic: one all-gather into and one reduce-scatter out of a [msg_bytes] tensor (the
    sequence-parallel region's activation), as `utils.comm` issues them."""
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    n, m = _sizes(msg_bytes, world)
    x = _int_data(n, device, 1000 + rank)
    shard = x[rank * m:(rank + 1) * m].clone()
    ref_full = torch.empty(n, dtype=x.dtype, device=device)
    ref_rs = torch.empty(m, dtype=x.dtype, device=device)
    state = {}

    def rccl():
        def run():
            _pg_all_gather(ref_full, shard, group)
            _pg_reduce_scatter(ref_rs, x, group)

        return Candidate("rccl", run)

    def xgmi(engine):
        def build():
            from .xgmi import XgmiCommunicator

            if "comm" not in state:
                state["comm"] = XgmiCommunicator(group, capacity_bytes=2 * n * 2 + (1 << 20), device=device,
                                                 timeout_s=timeout_s)
            c = state["comm"]
            c.gather_engine = engine
            full = torch.empty(n, dtype=x.dtype, device=device)
            rs = torch.empty(m, dtype=x.dtype, device=device)

            def run():
                c.all_gather_into(full, shard)
                c.reduce_scatter_into(rs, x)

            def verify():
                c.check()
                return bool(torch.equal(full, ref_full)) and bool(torch.equal(rs, ref_rs))

            last = engine == "dma" or "xgmi-dma" not in candidates
            return Candidate("xgmi-dma" if engine == "dma" else "xgmi", run, verify,
                             close=(lambda: state.pop("comm").close()) if last else None)

        return build

    out = {"rccl": rccl}
    if "xgmi" in candidates:
        out["xgmi"] = xgmi("kernel")
    if "xgmi-dma" in candidates:
        out["xgmi-dma"] = xgmi("dma")
    return out


def dp_builders(group, device, msg_bytes: int, timeout_s: float = None, candidates=CANDIDATES["dp"]):
    """Data-parallel traffic: one gradient-bucket reduce-scatter and one parameter all-gather of
    `msg_bytes`, on RCCL and on ZeRO's copy-engine path over shared flat buffers (the exact code
    the engine runs, parallel/xgmi_dp.py)."""
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    n, m = _sizes(msg_bytes, world)
    g = _int_data(n, device, 2000 + rank)
    p = _int_data(n, device, 3000)  # the all-gather input: every rank's slice of one buffer
    ref_rs = torch.empty(m, dtype=g.dtype, device=device)
    ref_ag = torch.empty(n, dtype=g.dtype, device=device)

    def rccl():
        def run():
            _pg_reduce_scatter(ref_rs, g, group)
            _pg_all_gather(ref_ag, p[rank * m:(rank + 1) * m], group)

        return Candidate("rccl", run)

    def xgmi_dma():
        from .xgmi_dp import XgmiZero

        z = XgmiZero(group, device, timeout_s=timeout_s)
        try:
            gbuf = z.alloc(n, torch.bfloat16, "grad")
            pbuf = z.alloc(n, torch.bfloat16, "param")
        except Exception:
            z.close()
            raise
        gbuf.copy_(g)
        out = torch.empty(m, dtype=g.dtype, device=device)
        ranges = [(r * m, (r + 1) * m) for r in range(world)]

        def run():
            pbuf.zero_()
            pbuf[rank * m:(rank + 1) * m].copy_(p[rank * m:(rank + 1) * m])
            z.reduce_scatter(gbuf, ranges, out).wait()
            z.all_gather(pbuf, ranges).wait()

        def verify():
            z.check()
            return bool(torch.equal(out, ref_rs)) and bool(torch.equal(pbuf, ref_ag))

        return Candidate("xgmi-dma", run, verify, close=z.close)

    out = {"rccl": rccl}
    if "xgmi-dma" in candidates:
        out["xgmi-dma"] = xgmi_dma
    return out


def select(kind: str, group, device, msg_bytes: int, timeout_s: float = None, warmup: int = 2, iters: int = 5,
           time_fn=None, candidates=None) -> tuple:
    """(choice, table) for `kind` in ("tp", "dp").  Off the GPU, or with one rank, or on a
    non-RCCL process group (gloo rehearsals), the only transport is the process group's own."""
    assert kind in CANDIDATES, kind
    dev = torch.device(device) if device is not None else torch.device("cpu")
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return "rccl", {}
    cands = tuple(candidates or CANDIDATES[kind])
    if dev.type != "cuda" and time_fn is None:
        return "rccl", {"rccl": {"us": None, "note": "CPU: the process group's backend is the only transport"}}
    if dist.get_backend(group) != "nccl" and time_fn is None and os.environ.get("DTG_TRANSPORT_CALIBRATE") != "1":
        # a gloo process group on GPUs is a rehearsal (ranks sharing one GPU): its timings say
        # nothing about a node, so it keeps the process group's collectives unless asked
        return "rccl", {"rccl": {"us": None, "note": "non-RCCL process group: not calibrated "
                                                     "(DTG_TRANSPORT_CALIBRATE=1 forces it)"}}
    builders = (tp_builders if kind == "tp" else dp_builders)(group, dev, msg_bytes, timeout_s, cands) \
        if time_fn is None else {c: (lambda c=c: Candidate(c, lambda: None)) for c in cands}
    table = measure(builders, group, dev, warmup, iters, time_fn=time_fn)
    table = {k: dict(v, msg_mib=round(msg_bytes / 2**20, 2)) for k, v in table.items()}
    return pick(table), table


def resolve(flag: str, kind: str, group, device, msg_bytes: int, timeout_s: float = None, log=None) -> tuple:
    """`--tp-comm` / `--dp-comm` value -> (transport, calibration table or None)."""
    if flag != "auto":
        return flag, None
    choice, table = select(kind, group, device, msg_bytes, timeout_s)
    _log_table(log, kind, msg_bytes, table, choice)
    return choice, table


# ------------------------------------------------------------------------------------------
# calibration in a child job (the trainer's `auto`)
# ------------------------------------------------------------------------------------------
CHILD_TIMEOUT = float(os.environ.get("DTG_TRANSPORT_CHILD_TIMEOUT", "180"))
_CHILD_SCRIPT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_transport_child.py")


def _log_table(log, kind, msg_bytes, table, choice):
    if log is None or not table:
        return
    rows = []
    for k, v in table.items():
        s = f"{k} {v.get('us')} us"
        if v.get("error"):
            s += f" ({v['error']})"
        elif v.get("note"):
            s += f" ({v['note']})"
        rows.append(s)
    log(f"{kind} transport calibration at {msg_bytes / 2**20:.1f} MiB: " + ", ".join(rows) + f" -> {choice}")


def _free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def child_command(world: int, spec: dict) -> list:
    """`torchrun --nproc-per-node world _transport_child.py <spec>` on this node's GPUs."""
    import json
    import sys

    stub = os.environ.get("DTG_TRANSPORT_CHILD_CMD")
    if stub:  # tests: a JSON argv that stands in for the child job
        return list(json.loads(stub))
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
            "--master-addr=127.0.0.1", f"--master-port={_free_port()}", _CHILD_SCRIPT, json.dumps(spec)]


def run_child(world: int, spec: dict, timeout: float) -> dict:
    """Run the calibration child job (own session, killed whole on timeout) -> its JSON record
    {"choice", "table"} or {"error", "stderr_tail"}."""
    import json
    import signal
    import subprocess

    drop = ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK", "ROLE_WORLD_SIZE",
            "MASTER_ADDR", "MASTER_PORT", "GROUP_WORLD_SIZE")
    env = {k: v for k, v in os.environ.items() if k not in drop and not k.startswith("TORCHELASTIC_")}
    try:
        pr = subprocess.Popen(child_command(world, spec), stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                              env=env, start_new_session=True)
    except Exception as e:  # noqa: BLE001
        return {"error": f"calibration child did not start: {e!r}"[:300]}
    try:
        out, err = pr.communicate(timeout=max(1.0, timeout))
    except subprocess.TimeoutExpired:
        try:
            os.killpg(pr.pid, signal.SIGKILL)
        except ProcessLookupError:
            pass
        out, err = pr.communicate()
        return {"error": f"calibration child timed out ({timeout:.0f} s)", "stderr_tail": (err or "")[-400:]}
    lines = [ln for ln in (out or "").splitlines() if ln.startswith("{")]
    if pr.returncode != 0 or not lines:
        return {"error": f"calibration child exited {pr.returncode}", "stderr_tail": (err or "")[-400:]}
    try:
        rec = json.loads(lines[-1])
    except ValueError as e:
        return {"error": f"calibration child printed no JSON record: {e}"}
    if rec.get("choice") not in CANDIDATES[spec["kind"]]:
        return {"error": f"calibration child picked {rec.get('choice')!r}"}
    return rec


def resolve_isolated(flag: str, kind: str, device, msg_bytes: int, mesh=(1, 0), timeout_s: float = None,
                     log=None, child_timeout: float = None) -> tuple:
    """`--tp-comm` / `--dp-comm` for the trainer: like `resolve`, but the measurement (and with it
    the xGMI library's first cross-device IPC contact) runs in a CHILD job on the same GPUs --
    `torchrun --nproc-per-node W parallel/_transport_child.py` started by rank 0 -- so a peer
    mapping that faults, or a collective that hangs, ends the child, never the training processes.
    Rank 0 broadcasts the child's pick; on any child failure or timeout every rank takes RCCL and
    the error is logged and returned in the table.  `mesh` = (k, axis) names the child's group:
    `make_mesh(k)[axis]` (k = 1: the whole world).  Collective over the default group.

    Off the GPU, on a non-RCCL group (gloo rehearsals) and on multi-node jobs (the child can only
    start this node's ranks) the process group's own collectives are used without measuring."""
    if flag != "auto":
        return flag, None
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return "rccl", {}
    dev = torch.device(device) if device is not None else torch.device("cpu")
    world = dist.get_world_size()
    forced = bool(os.environ.get("DTG_TRANSPORT_CHILD_CMD"))
    if not forced:
        note = None
        if dev.type != "cuda":
            note = "CPU: the process group's backend is the only transport"
        elif dist.get_backend() == "fake":
            note = "DTG_FAKE_WORLD rehearsal: no peers to calibrate against"
        elif dist.get_backend() != "nccl" and os.environ.get("DTG_TRANSPORT_CALIBRATE") != "1":
            note = "non-RCCL process group: not calibrated (DTG_TRANSPORT_CALIBRATE=1 forces it)"
        elif int(os.environ.get("LOCAL_WORLD_SIZE", world)) != world:
            note = "multi-node job: the calibration child only reaches this node's GPUs"
        if note is not None:
            table = {"rccl": {"us": None, "note": note}}
            _log_table(log, kind, msg_bytes, table, "rccl")
            return "rccl", table
    spec = {"kind": kind, "msg_bytes": int(msg_bytes), "mesh": [int(mesh[0]), int(mesh[1])],
            "timeout_s": timeout_s}
    box = [None]
    if dist.get_rank() == 0:
        box[0] = run_child(world, spec, CHILD_TIMEOUT if child_timeout is None else child_timeout)
    dist.broadcast_object_list(box, src=0)
    rec = box[0] or {"error": "no record"}
    if "error" in rec:
        table = {"rccl": {"us": None, "note": "fallback: calibration child failed"},
                 "child": {"us": None, "error": rec["error"] + (f" | {rec['stderr_tail'][-200:]}"
                                                                if rec.get("stderr_tail") else "")}}
        _log_table(log, kind, msg_bytes, table, "rccl")
        return "rccl", table
    _log_table(log, kind, msg_bytes, rec["table"], rec["choice"])
    return rec["choice"], rec["table"]


def child_main(argv) -> int:
    """The calibration child job: one rank per GPU, `select(kind)` on the requested group, rank 0
    prints {"choice", "table"}."""
    import json

    from ..utils.dist import init_distributed

    spec = json.loads(argv[0])
    # the trainer's own bootstrap: one GPU per rank over RCCL (or the DTG_SHARED_DEVICE rehearsal)
    _, _, _, dev = init_distributed()
    k, axis = spec["mesh"]
    group = None
    if k > 1:
        from .tensor_parallel import make_mesh

        group = make_mesh(k)[axis]
    choice, table = select(spec["kind"], group, dev, spec["msg_bytes"], spec.get("timeout_s"))
    if dist.get_rank() == 0:
        print(json.dumps({"choice": choice, "table": table}), flush=True)
    dist.barrier()
    dist.destroy_process_group()
    return 0


def tp_message_bytes(batch: int, seq: int, hidden: int, esz: int = 2) -> int:
    """Bytes of one sequence-parallel region's full activation [B*S, H] (the all-gather output)."""
    return int(batch) * int(seq) * int(hidden) * esz


__all__: List[str] = ["Candidate", "measure", "pick", "select", "resolve", "resolve_isolated", "tp_builders",
                      "dp_builders", "tp_message_bytes", "CANDIDATES"]
