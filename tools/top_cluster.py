#!/usr/bin/env python3
"""Cluster GPU monitor for MI355X nodes (reference top-cluster.py).

Every --poll-freq ms, in parallel per host, runs `amd-smi metric` (falls back to `rocm-smi`)
over ssh (or locally for `localhost`) and prints per-node and cluster means of GPU utilisation,
power as % of the cap, VRAM use and the number of GPU processes.  A hung job shows as power near
idle on every GPU (the reference's "~10% of the power limit" hang signature).

    python tools/top_cluster.py hosts            # hosts file, one host per line
    python tools/top_cluster.py localhost --once
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import json
import subprocess
import time


def _run(host: str, cmd: str) -> str:
    full = cmd if host in ("localhost", "127.0.0.1") else f"ssh -o BatchMode=yes {host} '{cmd}'"
    r = subprocess.run(full, shell=True, capture_output=True, text=True, timeout=30)
    return r.stdout


def _num(v):
    if isinstance(v, dict):
        v = v.get("value", v.get("current", 0))
    try:
        return float(str(v).split()[0])
    except (ValueError, IndexError):
        return 0.0


def parse_amd_smi(metric_json: str, process_json: str):
    """Returns a list of per-GPU dicts {util, power, power_cap, mem_used, mem_total, nprocs}."""
    gpus = []
    data = json.loads(metric_json) if metric_json.strip() else []
    if isinstance(data, dict):
        data = data.get("gpu_data", data.get("gpus", [data]))
    for g in data:
        usage = g.get("usage", {})
        power = g.get("power", {})
        mem = g.get("mem_usage", g.get("vram", {}))
        gpus.append({
            "util": _num(usage.get("gfx_activity", usage.get("gfx_usage", 0))),
            "power": _num(power.get("socket_power", power.get("current_socket_power", 0))),
            "power_cap": _num(power.get("power_limit", power.get("socket_power_limit", 0))) or 1400.0,
            "mem_used": _num(mem.get("used_vram", mem.get("vram_used", 0))),
            "mem_total": _num(mem.get("total_vram", mem.get("vram_total", 0))) or 288 * 1024.0,
            "nprocs": 0,
        })
    try:
        procs = json.loads(process_json) if process_json.strip() else []
        if isinstance(procs, list):
            for i, p in enumerate(procs):
                lst = p.get("process_list", [])
                if i < len(gpus):
                    gpus[i]["nprocs"] = len([x for x in lst if isinstance(x, dict) and x.get("process_info")])
    except json.JSONDecodeError:
        pass
    return gpus


def poll(host: str):
    m = _run(host, "amd-smi metric --usage --power --mem-usage --json 2>/dev/null")
    p = _run(host, "amd-smi process --json 2>/dev/null")
    try:
        return host, parse_amd_smi(m, p)
    except (json.JSONDecodeError, AttributeError, TypeError):
        return host, []


def summarize(gpus):
    if not gpus:
        return None
    n = len(gpus)
    return {
        "util": sum(g["util"] for g in gpus) / n,
        "power": 100 * sum(g["power"] / g["power_cap"] for g in gpus) / n,
        "mem": 100 * sum(g["mem_used"] / g["mem_total"] for g in gpus) / n,
        "nprocs": sum(g["nprocs"] for g in gpus),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("hosts", help="hosts file, or a single host name (localhost)")
    ap.add_argument("--poll-freq", type=int, default=1000, help="ms between polls")
    ap.add_argument("--once", action="store_true")
    a = ap.parse_args()
    try:
        with open(a.hosts) as fp:
            hosts = [l.strip() for l in fp if l.strip()]
    except FileNotFoundError:
        hosts = [a.hosts]
    while True:
        with cf.ThreadPoolExecutor(len(hosts)) as ex:
            res = dict(ex.map(poll, hosts))
        rows, allg = [], []
        for h in hosts:
            s = summarize(res.get(h, []))
            allg += res.get(h, [])
            rows.append((h, s))
        print(f"{'node':24s} {'util%':>7s} {'power%':>7s} {'mem%':>6s} {'procs':>6s}")
        for h, s in rows:
            if s is None:
                print(f"{h:24s} {'n/a':>7s}")
            else:
                print(f"{h:24s} {s['util']:7.1f} {s['power']:7.1f} {s['mem']:6.1f} {s['nprocs']:6d}")
        c = summarize(allg)
        if c:
            print(f"{'cluster':24s} {c['util']:7.1f} {c['power']:7.1f} {c['mem']:6.1f} {c['nprocs']:6d}")
            if c["power"] < 20 and c["nprocs"] > 0:
                print("WARNING: processes present but power ~idle -> likely hung collective (see diagnosing-errors/)")
        if a.once:
            break
        time.sleep(a.poll_freq / 1000)


if __name__ == "__main__":
    main()
