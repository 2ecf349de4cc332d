#!/usr/bin/env python3
"""Write TunableOp table variants that pin candidate hipBLASLt solutions for chosen shapes.

Input: `build/gemm_sustained` JSON lines (one per candidate solution, several specs) and the
committed table.  For k = 0..K-1 the variant `<out>/v<k>.csv` pins, for every spec in the
JSON, its k-th fastest candidate by sustained time (the other rows unchanged), so a bench run
per variant measures the candidates in the training step itself -- where the inputs arrive
cold from the producing kernels and the clock is the step's -- which neither TunableOp's short
bursts nor the back-to-back sustained loop sees.

    python tools/tunableop_variants.py sustained.jsonl --k 4 --out /tmp/tv
"""
import argparse
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TABLE = os.path.join(ROOT, "tunableop", "tunableop_results_partial.csv")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("jsonl")
    ap.add_argument("--k", type=int, default=4)
    ap.add_argument("--out", required=True)
    ap.add_argument("--table", default=TABLE)
    a = ap.parse_args()
    cands = {}
    for line in open(a.jsonl):
        line = line.strip()
        if not line.startswith("{"):
            continue
        r = json.loads(line)
        if r.get("sustained_ms") is None:
            continue
        cands.setdefault(r["spec"], []).append(r)
    for v in cands.values():
        v.sort(key=lambda r: r["sustained_ms"])
    base = open(a.table).read().splitlines()
    os.makedirs(a.out, exist_ok=True)
    for k in range(a.k):
        pins = {s: v[min(k, len(v) - 1)] for s, v in cands.items()}
        rows, seen = [], set()
        for line in base:
            f = line.split(",")
            if len(f) >= 4 and f[1] in pins:
                r = pins[f[1]]
                f[2] = "Default" if r.get("default") else f"Gemm_Hipblaslt_{r['index']}"
                f[3] = f"{r['sustained_ms']:.6f}"
                seen.add(f[1])
                line = ",".join(f)
            rows.append(line)
        for s, r in pins.items():
            if s not in seen:
                sol = "Default" if r.get("default") else f"Gemm_Hipblaslt_{r['index']}"
                rows.append(f"GemmTunableOp_BFloat16_TN,{s},{sol},{r['sustained_ms']:.6f}")
        path = os.path.join(a.out, f"v{k}.csv")
        with open(path, "w") as fp:
            fp.write("\n".join(rows) + "\n")
        print(path, {s: (r["index"], r["sustained_ms"], r.get("default")) for s, r in pins.items()})


if __name__ == "__main__":
    main()
