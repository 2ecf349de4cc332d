#!/usr/bin/env python3
"""Roofline table of one training step from the rocprofv3 --pmc passes of tools/step_pmc.sh.

    python tools/step_roofline.py gpurun_out/r3_s30/pmc [--steps 2] [--out table.md]

Per kernel family (hipBLASLt GEMMs grouped as one; dtg kernels by name), summed over all
dispatches of the profiled run and divided by `--steps` (warm-up + timed steps run by the pass),
or -- with `--window adamw_t` -- over exactly one step (between the last two optimizer launches):

  ms/step      kernel time from the pass-A dispatch timestamps (counter collection serialises
               dispatches, so each kernel ran alone on the GPU)
  mfma_busy    SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 256 CUs x 4 SIMDs): the
               fraction of SIMD cycles the matrix pipe was busy -- clock-independent
  eff. clock   MFMA-busy cycles each SIMD needed for the family's flops at 1,024 bf16 flops per
               SIMD-cycle, over the kernel time: the clock the GEMMs actually ran at (GEMMs only)
  GB r / w     FETCH_SIZE x --read-scale / WRITE_SIZE (KiB, L2 <-> fabric: HBM plus the MALL)
               per step.  FETCH_SIZE prices every read request that is not 32 B at 64 B, while
               gfx950's L2 fetches 128-B lines: on kernels whose bytes are known exactly the raw
               counter is half the algorithmic minimum (adamw_t: 32.1 GB raw vs 64.2 GB of p, g,
               m, v; swiglu_fwd: 15.0 vs 30.1 GB of gate/up), hence the default scale 2.
  TB/s         (read + write) / kernel time
"""
import argparse
import csv
import glob
import os
from collections import defaultdict

N_CU, N_XCD, SIMD = 256, 8, 4


def family(name):
    if "Cijk" in name:
        return "GEMM (hipBLASLt)"
    n = name.split("(")[0].replace("void ", "")
    return n.split("<")[0]


def load(d, window=None):
    """window = a kernel-name substring: keep only the dispatches after the second-to-last
    dispatch of that kernel up to and including the last one (one training step between two
    optimizer launches), in every pass (the passes run the same program)."""
    val = defaultdict(lambda: defaultdict(float))   # family -> counter@pass -> sum
    dur = defaultdict(float)                          # family -> ns (pass A timestamps)
    nd = defaultdict(set)
    for f in glob.glob(os.path.join(d, "*", "*counter_collection.csv")):
        pas = os.path.basename(os.path.dirname(f))
        seen = set()
        rows = list(csv.DictReader(open(f)))
        if window:
            ids = sorted({int(r["Dispatch_Id"]) for r in rows if window in r["Kernel_Name"]})
            lo, hi = ids[-2], ids[-1]
            rows = [r for r in rows if lo < int(r["Dispatch_Id"]) <= hi]
        for r in rows:
            fam = family(r["Kernel_Name"])
            val[fam][r["Counter_Name"] + "@" + pas] += float(r["Counter_Value"])
            key = (pas, r["Dispatch_Id"])
            if pas == "A" and key not in seen:
                seen.add(key)
                dur[fam] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
                nd[fam].add(r["Dispatch_Id"])
    return val, dur, nd


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--steps", type=int, default=2, help="steps in the run (ignored with --window)")
    ap.add_argument("--window", default=None, help="e.g. adamw_t: one step between the last two launches of this kernel")
    ap.add_argument("--flops-gemm", type=float, default=0.0,
                    help="GEMM flops per step (for the effective-clock column)")
    ap.add_argument("--top", type=int, default=18)
    ap.add_argument("--read-scale", type=float, default=2.0, help="bytes per FETCH_SIZE byte (see above)")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    val, dur, nd = load(a.dir, a.window)
    if a.window:
        a.steps = 1
    tot = sum(dur.values())
    rows = []
    for fam in sorted(dur, key=lambda f: -dur[f])[: a.top]:
        c = val[fam]
        ms = dur[fam] / 1e6 / a.steps
        grbm = c.get("GRBM_GUI_ACTIVE@A", 0.0)
        mb = c.get("SQ_VALU_MFMA_BUSY_CYCLES@A")
        busy = mb / (grbm / N_XCD * N_CU * SIMD) if (mb is not None and grbm > 0) else None
        rd = c.get("FETCH_SIZE@B")
        wr = c.get("WRITE_SIZE@C")
        gbr = rd * a.read_scale * 1024 / 1e9 / a.steps if rd is not None else None
        gbw = wr * 1024 / 1e9 / a.steps if wr is not None else None
        tbs = (gbr + gbw) / ms if (gbr is not None and gbw is not None and ms > 0) else None
        clk = None
        if fam.startswith("GEMM") and a.flops_gemm > 0 and busy:
            # busy SIMD-cycles needed = flops / 1024 per SIMD-cycle; over (time x SIMDs) = clock x busy
            clk = a.flops_gemm / 1024 / (N_CU * SIMD) / (busy * ms / 1e3) / 1e9
        rows.append((fam, len(nd[fam]) / a.steps, ms, 100 * dur[fam] / tot, busy, clk, gbr, gbw, tbs))
    f = lambda x, p=2: "-" if x is None else f"{x:.{p}f}"
    lines = ["| family | disp/step | ms/step | % | mfma_busy | eff. clock GHz | GB read | GB written | TB/s |",
             "|---|---:|---:|---:|---:|---:|---:|---:|---:|"]
    for fam, n, ms, pct, busy, clk, gbr, gbw, tbs in rows:
        lines.append(f"| `{fam}` | {n:.0f} | {ms:.2f} | {pct:.1f} | {f(busy)} | {f(clk)} | {f(gbr, 1)} | {f(gbw, 1)} | {f(tbs)} |")
    text = "\n".join(lines)
    print(text)
    if a.out:
        open(a.out, "w").write(text + "\n")


if __name__ == "__main__":
    main()
