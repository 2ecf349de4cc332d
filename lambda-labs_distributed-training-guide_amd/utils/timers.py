"""Phase timers.

`LocalTimer` reproduces the reference exactly: device synchronize on enter and exit, wall-clock
delta (its tok/s is a serialized step time).  `EventTimer` records HIP events instead and never
blocks the host; elapsed times are read lazily at log time, so the step loop keeps the GPU
queue full.  `make_timers(sync=...)` picks one; both expose avg_elapsed_ms()/reset().
"""
from __future__ import annotations

import time

import torch


class LocalTimer:
    def __init__(self, device: torch.device):
        self.synchronize = torch.cuda.synchronize if device.type == "cuda" else (lambda: None)
        self.measurements = []
        self.start_time = None

    def __enter__(self):
        self.synchronize()
        self.start_time = time.time()
        return self

    def __exit__(self, *exc):
        if exc[0] is None:
            self.synchronize()
            self.measurements.append(time.time() - self.start_time)
        self.start_time = None

    def avg_elapsed_ms(self):
        return 1000 * (sum(self.measurements) / len(self.measurements)) if self.measurements else 0.0

    def reset(self):
        self.measurements = []
        self.start_time = None


class EventTimer:
    """Asynchronous phase timer on HIP events (falls back to wall time on CPU)."""

    def __init__(self, device: torch.device):
        self.cuda = device.type == "cuda"
        self.pending = []
        self.done_ms = []
        self._start = None

    def __enter__(self):
        if self.cuda:
            self._start = torch.cuda.Event(enable_timing=True)
            self._start.record()
        else:
            self._start = time.perf_counter()
        return self

    def __exit__(self, *exc):
        if exc[0] is not None:
            return
        if self.cuda:
            end = torch.cuda.Event(enable_timing=True)
            end.record()
            self.pending.append((self._start, end))
        else:
            self.done_ms.append(1000 * (time.perf_counter() - self._start))

    def _drain(self):
        if self.pending:
            self.pending[-1][1].synchronize()
            self.done_ms.extend(s.elapsed_time(e) for s, e in self.pending)
            self.pending = []

    def avg_elapsed_ms(self):
        self._drain()
        return sum(self.done_ms) / len(self.done_ms) if self.done_ms else 0.0

    def reset(self):
        self._drain()
        self.done_ms = []


class _Ranged:
    """Wraps a timer with a roctx range (torch.cuda.nvtx maps to roctx on ROCm), so phases show
    up by name in rocprofv3 --marker-trace / Perfetto timelines."""

    def __init__(self, timer, name: str):
        self.timer, self.name = timer, name

    def __enter__(self):
        torch.cuda.nvtx.range_push(self.name)
        self.timer.__enter__()
        return self

    def __exit__(self, *exc):
        self.timer.__exit__(*exc)
        torch.cuda.nvtx.range_pop()

    def avg_elapsed_ms(self):
        return self.timer.avg_elapsed_ms()

    def reset(self):
        self.timer.reset()


def make_timers(device, names=("data", "forward", "backward", "update"), sync: bool = True, ranges: bool = False):
    cls = LocalTimer if sync else EventTimer
    timers = {k: cls(device) for k in names}
    if ranges and device.type == "cuda":
        timers = {k: _Ranged(t, k) for k, t in timers.items()}
    return timers
