#!/usr/bin/env python3
"""Summarise a rocprofv3 rocpd database (ROCm 7 default output): per-kernel time and, when the
run collected them, per-kernel PMC counter sums.

    python tools/rocpd_summary.py gpurun_out/prof/run_results.db [--top 20] [--match fa::]
"""
import argparse
import sqlite3
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--match", default="")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = list(c.execute("select name, count(*), sum(duration), avg(duration) from kernels group by name "
                          "order by sum(duration) desc"))
    total = sum(r[2] for r in rows) or 1
    print(f"| kernel | calls | total ms | avg us | % |\n|---|---:|---:|---:|---:|")
    for name, n, tot, avg in rows[: a.top]:
        if a.match and a.match not in name:
            continue
        short = name if len(name) < 90 else name[:87] + "..."
        print(f"| `{short}` | {n} | {tot / 1e6:.3f} | {avg / 1e3:.1f} | {100 * tot / total:.1f} |")
    try:
        pmc = list(c.execute("select kernel_name, counter_name, value from counters_collection"))
    except sqlite3.Error:
        pmc = []
    if pmc:
        agg = defaultdict(lambda: defaultdict(float))
        cnt = defaultdict(lambda: defaultdict(int))
        for k, cn, v in pmc:
            agg[k][cn] += v
            cnt[k][cn] += 1
        names = sorted({cn for k in agg for cn in agg[k]})
        print("\n| kernel | " + " | ".join(names) + " |\n|---|" + "---:|" * len(names))
        for k in agg:
            if a.match and a.match not in k:
                continue
            short = k if len(k) < 60 else k[:57] + "..."
            vals = [agg[k][cn] / max(1, cnt[k][cn]) for cn in names]
            print(f"| `{short}` | " + " | ".join(f"{v:.4g}" for v in vals) + " |")


if __name__ == "__main__":
    main()
