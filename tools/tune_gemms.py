#!/usr/bin/env python3
"""Offline GEMM tuning on one MI355X: tune the GEMM shapes a run recorded, one shape at a time,
saving the winners after every shape so that a time limit never loses finished work.

Two steps (the framework's runs read the committed table `tunableop/tunableop_results_partial.csv`):

    # 1. record: any training/bench run with DTG_TUNABLEOP_RECORD set lists the GEMM shapes the
    #    committed table lacks (dtg.utils.gemm_tuning.enable_tunableop)
    DTG_TUNABLEOP_RECORD=/tmp/untuned.csv python bench.py --model llama-2-7b --batch-size 10
    # 2. tune them (rewrites <out> after each shape), then merge into the committed table
    python tools/tune_gemms.py "/tmp/untuned*.csv" --out gpurun_out/tuned.csv --budget-s 600
    python tools/merge_tunableop.py tunableop/tunableop_results_partial.csv gpurun_out/tuned.csv

The tuning runs in a worker process; the parent (which never touches the GPU) prints progress,
and kills and restarts the worker past a shape that exceeds --shape-timeout-s (e.g. a head GEMM
over an odd 156,939-wide vocabulary where some library candidates are pathologically slow), so
one bad shape costs its timeout and nothing else.  Online tuning inside a training step
(`--tunableop tune`) does the same work, but a run killed by its time limit keeps none of it.
"""
import argparse
import glob
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _shapes(patterns, known):
    seen, out = set(), []
    for pat in patterns:
        for f in sorted(glob.glob(pat)):
            for line in open(f):
                parts = line.strip().split(",")
                if len(parts) < 2 or not parts[0].startswith("Gemm"):
                    continue
                key = (parts[0], parts[1])
                if key in seen or key in known:
                    continue
                seen.add(key)
                out.append(line.strip())
    return out


def _known(table):
    if not os.path.exists(table):
        return set()
    return {tuple(l.split(",")[:2]) for l in open(table) if l.startswith("Gemm")}


def _worker(shapes_file, results_file, max_tuning_ms, rotating_mb=0):
    """Tune every shape in shapes_file in order; after each, append its result line (JSON)."""
    # Compare every candidate's output with the default kernel's and drop the ones that differ:
    # without this TunableOp ranks on time alone, and one hipBLASLt solution for GPT-2's batched
    # attention-score GEMM (tn_1024_1024_64_B_96) returned values of order 1e33 -- NaN losses
    # (found by tools/check_tunableop.py, profiles/r2/s35/).
    # format "atol_rtol" (PyTorch 2.10): bf16 outputs of two correct kernels differ by rounding
    # (a few ulps of values ~sqrt(K)); a broken one is off by orders of magnitude
    os.environ.setdefault("PYTORCH_TUNABLEOP_NUMERICAL_CHECK", "1e-1_5e-2")
    import torch

    t = torch.cuda.tunable
    t.enable(True)
    t.set_filename(os.path.join(tempfile.gettempdir(), f"dtg_tune_{os.getpid()}.csv"), insert_device_ordinal=False)
    t.tuning_enable(True)
    t.set_max_tuning_duration(max_tuning_ms)
    t.set_max_tuning_iterations(50)
    if rotating_mb > 0:
        # candidates timed over a rotating set of operand copies larger than the caches: cold
        # inputs, as in a training step where each GEMM reads what another kernel just wrote
        t.set_rotating_buffer_size(rotating_mb)
    one = os.path.join(tempfile.gettempdir(), f"dtg_tune_one_{os.getpid()}.csv")
    for line in open(shapes_file).read().splitlines():
        with open(one, "w") as fp:
            fp.write(line + "\n")
        s = time.time()
        t.tune_gemm_in_file(one)
        torch.cuda.synchronize()
        key = tuple(line.split(",")[:2])
        best = next((list(r) for r in t.get_results() if (r[0], r[1]) == key), None)
        with open(results_file, "a") as fp:
            fp.write(json.dumps({"shape": line, "result": best, "s": round(time.time() - s, 1)}) + "\n")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("untuned", nargs="*", help="untuned-shape CSV files (globs ok)")
    ap.add_argument("--out", help="results CSV (rewritten after every shape)")
    ap.add_argument("--table", default=None, help="committed table; its shapes are skipped")
    ap.add_argument("--budget-s", type=float, default=600.0, help="stop starting new shapes after this")
    ap.add_argument("--shape-timeout-s", type=float, default=90.0)
    ap.add_argument("--max-tuning-ms", type=int, default=30)
    ap.add_argument("--rotating-mb", type=int, default=0, help="TunableOp rotating operand buffer (cold-cache timing)")
    ap.add_argument("--retune", action="store_true", help="tune shapes even if the committed table has them")
    ap.add_argument("--worker", nargs=2, metavar=("SHAPES", "RESULTS"), help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.worker:
        return _worker(args.worker[0], args.worker[1], args.max_tuning_ms, args.rotating_mb)

    table = args.table or os.path.join(ROOT, "tunableop", "tunableop_results_partial.csv")
    todo = _shapes(args.untuned, set() if args.retune else _known(table))
    print(f"[tune_gemms] {len(todo)} new GEMM shapes", flush=True)
    header = [l for l in open(table) if l.startswith("Validator")] if os.path.exists(table) else []
    work = tempfile.mkdtemp(prefix="dtg_tune_")
    results_file = os.path.join(work, "results.jsonl")
    open(results_file, "w").close()
    tuned, skipped = {}, []
    n_seen = 0
    t0 = last_print = time.time()
    while todo and time.time() - t0 < args.budget_s:
        shapes_file = os.path.join(work, "shapes.csv")
        with open(shapes_file, "w") as fp:
            fp.write("\n".join(todo) + "\n")
        proc = subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__), "--worker", shapes_file, results_file,
                                 "--max-tuning-ms", str(args.max_tuning_ms), "--rotating-mb", str(args.rotating_mb)])
        last = time.time()
        while True:
            time.sleep(1.0)
            lines = open(results_file).read().splitlines()
            for rec in map(json.loads, lines[n_seen:]):
                todo.remove(rec["shape"])
                r = rec["result"]
                if r:
                    tuned[tuple(r[:2])] = r
                print(f"[tune_gemms] {len(tuned)} done, {len(todo)} left: {rec['shape'].split(',')[1]} -> "
                      f"{r[2] if r else '?'} {float(r[3]) if r else 0:.4f} ms ({rec['s']}s)", flush=True)
                last = time.time()
            n_seen = len(lines)
            if args.out and tuned:
                tmp = args.out + ".tmp"
                with open(tmp, "w") as fp:
                    fp.write("".join(header) + "".join(",".join(str(x) for x in r) + "\n" for r in tuned.values()))
                os.replace(tmp, args.out)
            if proc.poll() is not None:
                break
            if time.time() - last > args.shape_timeout_s or time.time() - t0 > args.budget_s + args.shape_timeout_s:
                proc.kill()
                proc.wait()
                if todo and time.time() - last > args.shape_timeout_s:
                    bad = todo.pop(0)
                    skipped.append(bad)
                    print(f"[tune_gemms] skipped after {args.shape_timeout_s:.0f}s: {bad.split(',')[1]}", flush=True)
                break
            if time.time() - last_print > 30:
                last_print = time.time()
                print(f"[tune_gemms] ... {time.time() - t0:.0f}s, tuning {todo[0].split(',')[1] if todo else ''}",
                      flush=True)
        if proc.returncode not in (0, -9):
            # the worker died on its own (a fault, an abort): nothing more goes to the GPU
            print(f"[tune_gemms] worker exited {proc.returncode} on {todo[0].split(',')[1] if todo else '?'}; stopping",
                  flush=True)
            break
    print(f"[tune_gemms] tuned {len(tuned)}, skipped {len(skipped)}, untouched {len(todo)} "
          f"in {time.time() - t0:.0f}s -> {args.out}", flush=True)


if __name__ == "__main__":
    main()
