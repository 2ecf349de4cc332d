"""RCCL (torch's "nccl" backend on ROCm) environment preset and self-diagnosis.

The reference tried NCCL environment knobs on its 405B run and recorded that none helped
(/root/reference/05-training-llama-405b/launch.sh:18-20, README.md:230).  On an MI355X node the
relevant facts are different: the 8 GPUs are fully connected by point-to-point xGMI links, RCCL's
collectives are CU kernels that compete with the GEMMs they overlap, and the choice of transport
(P2P over xGMI vs shared memory vs network) decides the bandwidth.  So this module does two
things:

* `apply_preset(kind)` sets the environment a data-parallel training job on one MI355X node (or
  several) wants, without overriding anything the user exported.  Every knob is documented with
  why; `kind="none"` leaves the environment alone.
* `arm_log()` (before `init_process_group`) points RCCL's INIT/GRAPH info log at a per-process
  file, and `diagnose()` parses it afterwards into what RCCL actually built: version, ranks /
  nodes per communicator, channel count, and the transport of every ring/tree connection.  The
  bench attaches that record to its N > 1 JSON line, so a scaling number comes with its cause.
"""
from __future__ import annotations

import os
import re
import tempfile
from collections import Counter

# knob -> (value, reason).  Applied with setdefault semantics.
PRESETS = {
    "node": {
        # comm streams at high priority: bucket collectives issued during backward get scheduled
        # ahead of queued GEMM work instead of waiting behind it
        "TORCH_NCCL_HIGH_PRIORITY": ("1", "collectives overlapped with backward start promptly"),
        # record_stream on every collective input keeps gradient buckets alive until the caching
        # allocator sees the comm stream finish; the engines own their flat buffers for the
        # whole run, so the bookkeeping is pure overhead (the reference sets it for 405B)
        "TORCH_NCCL_AVOID_RECORD_STREAMS": ("1", "flat buckets live for the run; skip record_stream"),
        # ROCm's scratch reclaim can stall long-running RCCL kernels that use scratch
        "HSA_NO_SCRATCH_RECLAIM": ("1", "no scratch reclaim under persistent RCCL kernels"),
        # dmabuf IPC only on this fleet's driver: legacy IPC handles fail for RCCL P2P
        "HSA_ENABLE_IPC_MODE_LEGACY": ("0", "dmabuf IPC (required by the host driver)"),
    },
    "multinode": {
        "TORCH_NCCL_HIGH_PRIORITY": ("1", "as for one node"),
        "TORCH_NCCL_AVOID_RECORD_STREAMS": ("1", "as for one node"),
        "HSA_NO_SCRATCH_RECLAIM": ("1", "as for one node"),
        "HSA_ENABLE_IPC_MODE_LEGACY": ("0", "as for one node"),
        # rings may leave a node through a different NIC than they entered (the reference's
        # 405B launcher sets the same knob, launch.sh:18)
        "NCCL_CROSS_NIC": ("1", "let inter-node rings use any NIC pair"),
    },
}


def apply_preset(kind: str = "node", env=None) -> dict:
    """Set the preset's variables that are not already set; returns {name: value} applied."""
    env = os.environ if env is None else env
    if kind in (None, "", "none"):
        return {}
    applied = {}
    for k, (v, _why) in PRESETS[kind].items():
        if k not in env:
            env[k] = v
            applied[k] = v
    return applied


def arm_log(tag: str = "") -> str | None:
    """Before the first communicator exists: send RCCL's INIT/GRAPH/ENV info log to a file of
    this process (returned), unless the user already chose NCCL_DEBUG themselves (then None and
    their setting stands)."""
    if "NCCL_DEBUG" in os.environ:
        f = os.environ.get("NCCL_DEBUG_FILE")
        return f if f and "%" not in f else None
    path = os.path.join(tempfile.gettempdir(), f"dtg_rccl_{tag or os.getpid()}.log")
    try:
        os.remove(path)
    except OSError:
        pass
    os.environ["NCCL_DEBUG"] = "INFO"
    os.environ["NCCL_DEBUG_SUBSYS"] = "INIT,GRAPH,ENV"
    os.environ["NCCL_DEBUG_FILE"] = path
    return path


_RE_VERSION = re.compile(r"(?:RCCL|NCCL) version[ :]+([0-9][0-9A-Za-z.+\-_]*)")
_RE_CHANNEL = re.compile(r"Channel (\d+)/(\d+) :")
_RE_VIA = re.compile(r"Channel \d+/\d+ : (\d+)\[[^\]]*\] -> (\d+)\[[^\]]*\] (?:\[\w+\] )?via (\S+)")
_RE_COMM = re.compile(r"comm (0x[0-9a-f]+) rank (\d+) nRanks (\d+) nNodes (\d+) localRanks (\d+)")
_RE_COMM2 = re.compile(r"comm (0x[0-9a-f]+) rank (\d+) nranks (\d+) cudaDev (\d+)")
_RE_COLLCH = re.compile(r"(\d+) coll channels")
_RE_P2PCH = re.compile(r"(\d+) p2p channels per peer")


def parse_log(text: str) -> dict:
    """What RCCL built, from its INFO log: version, communicators (nRanks / nNodes), channel
    count, connection transports ({"P2P/IPC": n, "SHM": m, ...})."""
    version = None
    m = _RE_VERSION.search(text)
    if m:
        version = m.group(1)
    comms = {}
    for m in _RE_COMM.finditer(text):
        comms[m.group(1)] = {"rank": int(m.group(2)), "nranks": int(m.group(3)), "nnodes": int(m.group(4)),
                             "local_ranks": int(m.group(5))}
    for m in _RE_COMM2.finditer(text):
        comms.setdefault(m.group(1), {"rank": int(m.group(2)), "nranks": int(m.group(3)), "device": int(m.group(4))})
    nch = [int(m.group(2)) for m in _RE_CHANNEL.finditer(text)]
    via = Counter(m.group(3) for m in _RE_VIA.finditer(text))
    coll = [int(m.group(1)) for m in _RE_COLLCH.finditer(text)]
    p2p = [int(m.group(1)) for m in _RE_P2PCH.finditer(text)]
    return {
        "version": version,
        "communicators": list(comms.values()),
        "channels_max": max(nch) if nch else None,
        "coll_channels": sorted(set(coll)) or None,
        "p2p_channels_per_peer": sorted(set(p2p)) or None,
        "transports": dict(via),
    }


def env_snapshot() -> dict:
    """The NCCL_* / RCCL_* / HSA_* / TORCH_NCCL_* variables of this process."""
    keep = ("NCCL_", "RCCL_", "HSA_", "TORCH_NCCL_", "GPU_MAX_HW_QUEUES")
    return {k: v for k, v in sorted(os.environ.items()) if k.startswith(keep)}


def library_version() -> str | None:
    try:
        import torch

        v = torch.cuda.nccl.version()
        return ".".join(str(x) for x in v) if isinstance(v, tuple) else str(v)
    except Exception:
        return None


def diagnose(log_path: str | None) -> dict:
    """Version + environment + the parsed log (if one was captured)."""
    rec = {"library_version": library_version(), "env": env_snapshot(), "log": None}
    if log_path and os.path.exists(log_path):
        with open(log_path, errors="replace") as fp:
            rec["log"] = parse_log(fp.read())
        rec["log_file"] = log_path
    return rec
