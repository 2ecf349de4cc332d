#!/usr/bin/env python3
"""Per-kernel hardware-counter table from rocprofv3 --pmc CSV passes (tools/fa_pmc.sh).

    python tools/pmc_summary.py gpurun_out/r2_s17/llama8b [--match fa::]

Counters are summed over every dispatch of a kernel in each pass (each pass is a separate run
of the same program), then combined into the ratios that matter for an MFMA kernel:

  mfma_busy   SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs * CUs * 4 SIMDs)
              -- fraction of SIMD cycles the matrix pipe was busy (GRBM sums the 8 XCDs)
  wait/active/idle  SQ_WAIT_ANY, SQ_ACTIVE_INST_ANY, SQ_WAIT_INST_ANY over SQ_WAVE_CYCLES
              (quad-cycles; the three partition a wave's life)
  lds_wait    SQ_WAIT_INST_LDS / SQ_WAVE_CYCLES  (LDS-issue stalls)
  bank_conf   SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE  (extra LDS cycles per LDS-array cycle)
  valu/mfma   vector instructions per MFMA instruction
  GB          FETCH_SIZE (KiB) summed -> bytes fetched from HBM per dispatch
"""
import argparse
import csv
import glob
import os
from collections import defaultdict

N_CU = 256


def load(d, match):
    per = defaultdict(lambda: defaultdict(float))
    ndisp = defaultdict(lambda: defaultdict(set))
    for f in glob.glob(os.path.join(d, "*", "*counter_collection.csv")):
        pas = os.path.basename(os.path.dirname(f))
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if match and match not in k:
                continue
            per[k][r["Counter_Name"] + "@" + pas] += float(r["Counter_Value"])
            ndisp[k][pas].add(r["Dispatch_Id"])
    return per, ndisp


def short(k):
    k = k.split("(")[0]
    return k.replace("void ", "").replace("dtg::fa::", "")


def ctr(c, name):
    vals = [v for key, v in c.items() if key.split("@")[0] == name]
    return vals[0] if vals else None


def ctr_in(c, name, pas):
    return c.get(name + "@" + pas)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--match", default="fa::")
    a = ap.parse_args()
    per, nd = load(a.dir, a.match)
    print("| kernel | disp | mfma_busy | active | wait | stall | lds_wait | bank_conf | valu/mfma | GB/disp |")
    print("|---|---:|---:|---:|---:|---:|---:|---:|---:|---:|")
    for k, c in sorted(per.items()):
        n = max(len(s) for s in nd[k].values())
        pa = [p for p in nd[k] if ctr_in(c, "SQ_WAVE_CYCLES", p) is not None]
        pas = pa[0] if pa else None
        gui = ctr_in(c, "GRBM_GUI_ACTIVE", pas) if pas else None
        mb = ctr_in(c, "SQ_VALU_MFMA_BUSY_CYCLES", pas) if pas else None
        wc = ctr_in(c, "SQ_WAVE_CYCLES", pas) if pas else None

        def frac(x, y):
            return f"{x / y:.2f}" if (x is not None and y) else "-"

        busy = frac(mb, (gui / 8) * N_CU * 4) if (mb is not None and gui) else "-"
        act = frac(ctr_in(c, "SQ_ACTIVE_INST_ANY", pas), wc) if pas else "-"
        wait = frac(ctr_in(c, "SQ_WAIT_ANY", pas), wc) if pas else "-"
        stall = frac(ctr_in(c, "SQ_WAIT_INST_ANY", pas), wc) if pas else "-"
        ldsw = frac(ctr_in(c, "SQ_WAIT_INST_LDS", pas), wc) if pas else "-"
        bank = frac(ctr(c, "SQ_LDS_BANK_CONFLICT"), ctr(c, "SQ_LDS_IDX_ACTIVE"))
        vm = frac(ctr(c, "SQ_INSTS_VALU"), ctr(c, "SQ_INSTS_MFMA"))
        fs = ctr(c, "FETCH_SIZE")
        gb = f"{fs * 1024 / n / 1e9:.3f}" if fs is not None else "-"
        print(f"| `{short(k)}` | {n} | {busy} | {act} | {wait} | {stall} | {ldsw} | {bank} | {vm} | {gb} |")


if __name__ == "__main__":
    main()
