#!/usr/bin/env python3
"""Vocab-parallel loss head: is any collective waited on between the chunks?

From a rocprofv3 --kernel-trace CSV of one tensor-parallel rank, take every forward's loss-head
region (ce_stats_kernel ... ce_grad_kernel per chunk) and report, per chunk j:

  * whether chunk j+1's logits GEMM was issued (started) BEFORE chunk j's gradient kernel
    (the software pipeline: chunk j's stats gather in flight under the next GEMM);
  * how much of chunk j's stats all-gather (the xGMI barrier / gather kernels between
    ce_stats(j) and ce_grad(j)) overlapped a GEMM.

    python tools/ce_overlap.py gpurun_out/r3_s05/trace/r0
"""
import argparse
import csv
import glob
import os


def load(d):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    return sorted(rows)


def is_gemm(n):
    return n.startswith("Custom_Cijk") or n.startswith("Cijk")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    a = ap.parse_args()
    ks = load(a.dir)
    stats = [i for i, k in enumerate(ks) if "ce_stats_kernel" in k[2]]
    grads = [i for i, k in enumerate(ks) if "ce_grad_kernel" in k[2]]
    gemms = [k for k in ks if is_gemm(k[2])]
    print(f"{len(ks)} kernels, {len(stats)} ce_stats, {len(grads)} ce_grad")
    pipelined = total = 0
    overlap_ns = coll_ns = 0
    for si in stats:
        s_end = ks[si][1]
        gi = next((g for g in grads if g > si), None)
        if gi is None:
            continue
        nxt = next((j for j in range(si + 1, len(ks)) if "ce_stats_kernel" in ks[j][2]), None)
        total += 1
        # the next chunk's GEMM starts before this chunk's gradient kernel
        if nxt is not None and nxt < gi:
            pipelined += 1
        # collective kernels of this chunk: xgmi barrier / gather kernels between stats and grad
        coll = [k for k in ks[si + 1:gi] if "xgmi" in k[2] or "barrier_kernel" in k[2] or "all_gather_kernel" in k[2]]
        for c0, c1, _ in coll:
            coll_ns += c1 - c0
            for g0, g1, _ in gemms:
                lo, hi = max(c0, g0), min(c1, g1)
                if lo < hi:
                    overlap_ns += hi - lo
    print(f"chunks with the next chunk's stats issued before this chunk's gradient: {pipelined} / {total}")
    if coll_ns:
        print(f"stats-gather kernel time {coll_ns / 1e3:.1f} us, of which under a GEMM {overlap_ns / 1e3:.1f} us "
              f"({100 * overlap_ns / coll_ns:.0f} %)")


if __name__ == "__main__":
    main()
