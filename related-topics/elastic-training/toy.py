#!/usr/bin/env python3
"""Fault-injection toy for elastic restarts.  CPU only (gloo), no GPU needed.

Every step each rank draws a random number and raises with probability --fail-prob; torchrun
(`--max-restarts N`) then restarts ALL workers, which resume from `toy-state.json` (written by
rank 0 between two barriers).  RNG is reseeded from rank + world_size * num_steps after a
restart, so a restarted job does not replay the same failure.

    torchrun --nnodes 1 --nproc-per-node 4 --max-restarts 3 toy.py
"""
import argparse
import datetime
import json
import os
import random
import time

import torch.distributed as dist
from torch.distributed.elastic.multiprocessing.errors import record


@record
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--fail-prob", type=float, default=0.001)
    ap.add_argument("--state", default="./toy-state.json")
    ap.add_argument("--sleep", type=float, default=0.0)
    ap.add_argument("--fail-at-step", type=int, default=-1, help="deterministic failure of rank 1 on the first attempt")
    ap.add_argument("--pg-timeout", type=float, default=60.0, help="process-group timeout (s)")
    a = ap.parse_args()
    # a bounded rendezvous/connect: a worker whose mesh connect fails must exit (and let torchrun
    # restart the group) instead of waiting out the 30-minute default
    timeout = datetime.timedelta(seconds=a.pg_timeout)
    if os.environ.get("TORCHELASTIC_USE_AGENT_STORE") == "True":
        # torchrun keeps ONE agent-hosted TCPStore for every restart of the worker group, and
        # init_process_group's env:// path adds no per-attempt prefix: gloo's full-mesh
        # bootstrap then finds a peer's listening address from a previous attempt already in
        # the store, connects to a dead port ("Connection refused") and the failed attempt
        # leaves stale keys for the next one.  Keys of attempt N live under attempt_N instead.
        store = dist.TCPStore(os.environ["MASTER_ADDR"], int(os.environ["MASTER_PORT"]),
                              int(os.environ["WORLD_SIZE"]), is_master=False, timeout=timeout)
        store = dist.PrefixStore(f"toy/attempt_{os.environ.get('TORCHELASTIC_RESTART_COUNT', '0')}", store)
        dist.init_process_group("gloo", store=store, rank=int(os.environ["RANK"]),
                                world_size=int(os.environ["WORLD_SIZE"]), timeout=timeout)
    else:
        dist.init_process_group("gloo", timeout=timeout)
    rank, world = dist.get_rank(), dist.get_world_size()
    state = {"num_steps": 0}
    if os.path.exists(a.state):
        with open(a.state) as fp:
            state = json.load(fp)
    random.seed(rank + world * state["num_steps"])
    print(f"[rank {rank}] starting at step {state['num_steps']} (restart count {os.environ.get('TORCHELASTIC_RESTART_COUNT', 0)})", flush=True)
    while state["num_steps"] < a.steps:
        first_attempt = os.environ.get("TORCHELASTIC_RESTART_COUNT", "0") == "0"
        if state["num_steps"] == a.fail_at_step and rank == min(1, world - 1) and first_attempt:
            raise ValueError(f"rank {rank} deterministic failure at step {state['num_steps']}")
        if random.random() < a.fail_prob:
            raise ValueError(f"rank {rank} injected failure at step {state['num_steps']}")
        time.sleep(a.sleep)
        state["num_steps"] += 1
        dist.barrier()
        if rank == 0:
            with open(a.state, "w") as fp:
                json.dump(state, fp)
        dist.barrier()
    if rank == 0:
        print(f"finished {state['num_steps']} steps", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
