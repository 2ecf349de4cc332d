#!/usr/bin/env python3
"""How many copies run at once, from rocprofv3 --memory-copy-trace CSVs (and, with
--kernels, blit kernels of the kernel trace: ROCclr may run device-to-device copies as
`__amd_rocclr_copyBuffer` kernels instead of SDMA transfers).

    python tools/copy_concurrency.py gpurun_out/r3_s02/trace/r0 [--kernels]

Prints the number of copy intervals, the maximum overlap and the time spent at each overlap
level (a serialized issue shows max 1; the per-peer-stream DMA path should reach >= 4).
"""
import argparse
import csv
import glob
import os
from collections import defaultdict


def intervals(d, kernels):
    out = []
    for f in glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            out.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy:" + r.get("Direction", "?")))
    if kernels:
        for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if "copyBuffer" in r["Kernel_Name"]:
                    out.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "blit"))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--kernels", action="store_true")
    a = ap.parse_args()
    iv = intervals(a.dir, a.kernels)
    ev = sorted([(s, 1) for s, e, _ in iv] + [(e, -1) for s, e, _ in iv])
    cur, best, last = 0, 0, None
    at = defaultdict(int)
    for t, d in ev:
        if last is not None and cur > 0:
            at[cur] += t - last
        cur += d
        best = max(best, cur)
        last = t
    kinds = defaultdict(int)
    for _, _, k in iv:
        kinds[k] += 1
    print(f"{len(iv)} copy intervals {dict(kinds)}; max concurrent = {best}")
    tot = sum(at.values()) or 1
    for k in sorted(at):
        print(f"  {k} at once: {at[k] / 1e3:10.1f} us ({100 * at[k] / tot:5.1f} %)")


if __name__ == "__main__":
    main()
