#!/usr/bin/env python3
"""Per-step GPU busy time vs wall time from a rocprofv3 --kernel-trace CSV.

    rocprofv3 --kernel-trace -d gpurun_out/st -o run --output-format csv -- \
        python3 bench.py --steps 5 --warmup 2 --fsdp-mem-steps 0
    python tools/step_gaps.py gpurun_out/st [--marker adamw_kernel]

Steps are delimited by the optimizer kernel (one launch per step).  For every step window:
wall = marker-to-marker span, busy = union of kernel intervals (any stream), idle = the rest
(launch gaps, host syncs, allocator stalls).  Also prints the per-step kernel-time table of the
last window, grouped by kernel family.
"""
import argparse
import csv
import glob
import os
import re
from collections import defaultdict


def family(name):
    n = name.split("(")[0].replace("void ", "")
    if n.startswith("Custom_Cijk") or n.startswith("Cijk"):
        return "GEMM (hipBLASLt)"
    n = re.sub(r"<.*", "", n)
    return n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--marker", default="adamw_kernel")
    ap.add_argument("--sequence", default=None, help="write the last step's ordered kernel list (us, name) here")
    a = ap.parse_args()
    rows = []
    for f in glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows))
    marks = [e for s, e, n in ks if a.marker in n]
    print(f"{len(ks)} kernels, {len(marks)} '{a.marker}' markers")
    print("| step | wall ms | busy ms | idle ms | kernels |")
    print("|---:|---:|---:|---:|---:|")
    last = None
    for i in range(1, len(marks)):
        lo, hi = marks[i - 1], marks[i]
        iv = [(max(s, lo), min(e, hi), n) for s, e, n in ks if e > lo and s < hi]
        busy, cur_s, cur_e = 0, None, None
        for s, e, _ in sorted(iv):
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    busy += cur_e - cur_s
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        if cur_e is not None:
            busy += cur_e - cur_s
        wall = hi - lo
        print(f"| {i} | {wall / 1e6:.1f} | {busy / 1e6:.1f} | {(wall - busy) / 1e6:.1f} | {len(iv)} |")
        last = iv
    if last:
        fam = defaultdict(lambda: [0, 0])
        for s, e, n in last:
            fam[family(n)][0] += e - s
            fam[family(n)][1] += 1
        tot = sum(v[0] for v in fam.values())
        print("\nlast step, kernel time by family:\n")
        print("| family | calls | ms | % |")
        print("|---|---:|---:|---:|")
        for k, (t, c) in sorted(fam.items(), key=lambda kv: -kv[1][0]):
            print(f"| `{k[:70]}` | {c} | {t / 1e6:.2f} | {100 * t / tot:.1f} |")
        if a.sequence:
            with open(a.sequence, "w") as fp:
                for s, e, n in sorted(last):
                    fp.write(f"{(e - s) / 1e3:10.1f}  {n.split('(')[0][:150]}\n")


if __name__ == "__main__":
    main()
