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


def load(f):
    rows = []
    for r in csv.DictReader(open(f)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    return sorted(rows)


def is_gemm(n):
    return n.startswith("Custom_Cijk") or n.startswith("Cijk")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    a = ap.parse_args()
    # one kernel-trace CSV per process (rocprofv3 -o %pid%_run): each rank analysed on its own
    for f in sorted(glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True)):
        print(f"== {os.path.relpath(f, a.dir)}")
        analyse(load(f))


def analyse(ks):
    stats = [i for i, k in enumerate(ks) if "ce_stats_kernel" in k[2]]
    grads = [i for i, k in enumerate(ks) if "ce_grad_kernel" in k[2]]
    gemms = [k for k in ks if is_gemm(k[2])]
    print(f"{len(ks)} kernels, {len(stats)} ce_stats, {len(grads)} ce_grad")
    pipelined = total = 0
    overlap_ns = coll_ns = 0
    # the k-th stats kernel belongs to the k-th gradient kernel (chunks run in order); with the
    # pipeline, stats(j + 1) is issued before grad(j)
    for k, (si, gi) in enumerate(zip(stats, grads)):
        if gi < si:
            continue
        total += 1
        if k + 1 < len(stats) and stats[k + 1] < gi:  # (a forward's last chunk has no successor)
            pipelined += 1
        # collective kernels of this chunk: xgmi barrier / gather kernels between stats and grad
        coll = [c for c in ks[si + 1:gi] if "xgmi" in c[2] or "barrier_kernel" in c[2] or "all_gather_kernel" in c[2]]
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
