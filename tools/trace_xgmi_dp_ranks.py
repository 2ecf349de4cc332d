#!/usr/bin/env python3
"""Kernel trace of ONE rank of a multi-rank ZeRO run over the xGMI copy engines (VERDICT r3 #2:
"a rocprofv3 trace of a 4-rank shared-GPU step shows no RCCL kernels and only barrier and
reduce kernels on CUs during the overlap").

This launcher never touches the GPU itself: it starts `world` ranks of bench.py sharing the box's
GPU (DTG_SHARED_DEVICE=1, gloo bootstrap, `--dp-comm xgmi-dma`), rank 0 as the program of
`rocprofv3 --kernel-trace` (the profiler sees only that process), the others plain, and waits.

    python tools/trace_xgmi_dp_ranks.py --world 4 --out gpurun_out/r4_s28/trace
"""
import argparse
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=4)
    ap.add_argument("--out", required=True)
    ap.add_argument("--model", default="llama-3.2-3b")
    ap.add_argument("--steps", type=int, default=3)
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    port = free_port()
    bench = [os.path.join(ROOT, "bench.py"), "--gpus", str(a.world), "--backend", "gloo", "--model", a.model,
             "--batch-size", "2", "--steps", str(a.steps), "--warmup", "2", "--ref-steps", "0", "--fsdp-mem-steps", "0",
             "--coll-sweep-mb", "", "--bucket-sweep-mb", "", "--xgmi-child", "0", "--dp-comm", "xgmi-dma",
             "--rccl-preset", "none"]
    procs = []
    for r in range(a.world):
        env = dict(os.environ, DTG_SHARED_DEVICE="1", RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(a.world),
                   LOCAL_WORLD_SIZE=str(a.world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        if r == 0:
            cmd = ["rocprofv3", "--kernel-trace", "--stats", "-d", a.out, "-o", "rank0", "--", sys.executable] + bench
        else:
            cmd = [sys.executable] + bench
        log = open(os.path.join(a.out, f"rank{r}.log"), "w")
        procs.append((subprocess.Popen(cmd, cwd=ROOT, env=env, stdout=log, stderr=subprocess.STDOUT), log))
    rc = 0
    for p, log in procs:
        try:
            rc |= p.wait(timeout=600)
        except subprocess.TimeoutExpired:
            p.kill()
            rc |= 124
        log.close()
    print(f"ranks done rc={rc}", flush=True)
    return rc


if __name__ == "__main__":
    sys.exit(main())
