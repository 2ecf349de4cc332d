#!/usr/bin/env python3
"""Re-rank TunableOp's GEMM candidates under SUSTAINED load.

TunableOp times every candidate solution in short warm bursts (tens of ms, operands in cache),
where the chip runs at boost clocks.  In a training step the GEMMs run back to back for hundreds
of ms at power-limited clocks (profiles/r3/s30: ~1.7-1.8 GHz effective): the step's gate_up
forward GEMM takes 2.58 ms where its tuning burst measured 1.79 ms.  A solution that moves fewer
bytes or issues less work per FLOP can win under that limit while losing the burst.

    # 1. list: tune each shape with PYTORCH_TUNABLEOP_VERBOSE=3 and keep every candidate's burst time
    python tools/tunableop_sustained.py list --out gpurun_out/cands.json
    # 2. time the top-k candidates of each shape in a sustained loop (one child per candidate rank,
    #    the committed table with that rank's solutions substituted)
    python tools/tunableop_sustained.py time --cands gpurun_out/cands.json --top 4 --out gpurun_out/sustained.jsonl

Round 1's tools/gemm_sustained.cpp swept every hipBLASLt solution of the system library the same
way (profiles/r1: defaults within noise of the best, 32x32-MFMA solutions 13-17 % slower); this
tool ranks what PyTorch's own bundled library offers through TunableOp, i.e. exactly the
solutions a table entry can pin.

Shapes: the Llama-3-8B bench step's TN GEMMs at T = 16384 (key "tn_m_n_k": C[n, m] = A[n, k] B[m, k]^T).
"""
import argparse
import json
import os
import re
import subprocess
import sys
import tempfile
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
TABLE = os.path.join(ROOT, "tunableop", "tunableop_results_partial.csv")

STEP_SHAPES = {  # name: (m, n, k)
    "qkv_fwd": (6144, 16384, 4096), "o_fwd": (4096, 16384, 4096), "gu_fwd": (28672, 16384, 4096),
    "down_fwd": (4096, 16384, 14336),
    "qkv_dx": (4096, 16384, 6144), "gu_dx": (4096, 16384, 28672), "down_dx": (14336, 16384, 4096),
    "qkv_dw": (4096, 6144, 16384), "o_dw": (4096, 4096, 16384), "gu_dw": (4096, 28672, 16384),
    "down_dw": (14336, 4096, 16384),
}


def key_of(m, n, k):
    return f"tn_{m}_{n}_{k}_ld_{k}_{k}_{m}"


def operands(m, n, k, copies=1):
    import torch

    g = torch.Generator(device="cuda").manual_seed(0)
    return [(torch.randn(n, k, device="cuda", dtype=torch.bfloat16, generator=g),
             torch.randn(m, k, device="cuda", dtype=torch.bfloat16, generator=g)) for _ in range(copies)]


def cmd_list(a):
    """Tune every shape from scratch (verbose) and parse each candidate's burst time."""
    log = a.out + ".log"
    env = dict(os.environ, PYTORCH_TUNABLEOP_VERBOSE="3", PYTORCH_TUNABLEOP_VERBOSE_FILENAME="out")
    with open(log, "w") as fp:
        subprocess.run([sys.executable, "-u", os.path.abspath(__file__), "_tune", "--only", a.only or ""],
                       env=env, stdout=fp, stderr=subprocess.STDOUT, check=True)
    text = open(log).read()
    cands = parse_candidates(text)
    json.dump(cands, open(a.out, "w"), indent=1)
    for k, v in cands.items():
        print(k, len(v), v[:3], flush=True)


def parse_candidates(text):
    """{param key: [(solution, ms), ...] fastest first} from TunableOp's verbose tuning log."""
    # PyTorch 2.10's log: a quick first-iteration screen drops most candidates ("skip slow
    # instance"); each survivor gets one line
    #   ├──tuning using warmup iters 0 [0 ms] and tuning iters 30 [8.39 ms] instance id=0, <op>(<key>) <solution>
    # whose bracket is the total of its tuning iterations.
    cands = {}
    pat = re.compile(r"tuning iters (\d+) \[([0-9.]+) ms\] instance id=\d+, \w+\((tn_[0-9_ld]+)\) (\S+)")
    for line in text.splitlines():
        s = pat.search(line)
        if s:
            ms = float(s.group(2)) / max(1, int(s.group(1)))
            d = cands.setdefault(s.group(3), {})
            sol = s.group(4)
            if sol not in d or ms < d[sol]:
                d[sol] = round(ms, 5)
    return {k: sorted(v.items(), key=lambda x: x[1]) for k, v in cands.items() if v}


def _tune(a):
    import torch

    t = torch.cuda.tunable
    t.enable(True)
    t.set_filename(os.path.join(tempfile.gettempdir(), f"dtg_sustained_{os.getpid()}.csv"), insert_device_ordinal=False)
    t.tuning_enable(True)
    t.set_max_tuning_duration(30)
    t.set_max_tuning_iterations(30)
    for name, (m, n, k) in STEP_SHAPES.items():
        if a.only and name not in a.only.split(","):
            continue
        print(f"### shape {name} {key_of(m, n, k)}", flush=True)
        (x, w), = operands(m, n, k)
        torch.mm(x, w.t())
        torch.cuda.synchronize()
        del x, w
    print("### results", flush=True)
    for r in t.get_results():
        print("RESULT", ",".join(str(v) for v in r), flush=True)


def _time_child(a):
    """Sustained timing of every shape under the table in PYTORCH_TUNABLEOP_FILENAME."""
    import torch

    t = torch.cuda.tunable
    t.enable(True)
    t.tuning_enable(False)
    t.read_file(a.table)
    out = []
    for name, (m, n, k) in STEP_SHAPES.items():
        if a.only and name not in a.only.split(","):
            continue
        ops = operands(m, n, k, copies=2)  # alternate two operand sets (~0.3-1.6 GB): no L2 reuse
        c = torch.empty(n, m, device="cuda", dtype=torch.bfloat16)
        for i in range(20):
            x, w = ops[i % 2]
            torch.mm(x, w.t(), out=c)
        torch.cuda.synchronize()
        # sustained: >= a.seconds of back-to-back GEMMs, timed by events around the second half
        s0 = time.time()
        n_it = 0
        while time.time() - s0 < a.seconds / 2:
            for i in range(10):
                x, w = ops[i % 2]
                torch.mm(x, w.t(), out=c)
            n_it += 10
            torch.cuda.synchronize()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        for i in range(n_it):
            x, w = ops[i % 2]
            torch.mm(x, w.t(), out=c)
        ev1.record()
        torch.cuda.synchronize()
        ms = ev0.elapsed_time(ev1) / n_it
        out.append({"shape": name, "key": key_of(m, n, k), "ms": round(ms, 4),
                    "TFLOPs": round(2.0 * m * n * k / ms / 1e9, 1), "iters": n_it})
        print(json.dumps(out[-1]), flush=True)
        del ops, c
        torch.cuda.empty_cache()


def cmd_time(a):
    cands = json.load(open(a.cands))
    base = [l for l in open(TABLE)]
    committed = {tuple(l.split(",")[:2]): l.split(",")[2] for l in base if l.startswith("Gemm")}
    res = open(a.out, "a")
    for rank in range(-1, a.top):
        # rank -1: the committed table as it is
        lines, label = [], {}
        for l in base:
            parts = l.rstrip("\n").split(",")
            if l.startswith("GemmTunableOp_BFloat16_TN") and rank >= 0 and parts[1] in cands:
                cs = cands[parts[1]]
                if rank < len(cs):
                    parts[2] = cs[rank][0]
            if l.startswith("Gemm"):
                label[parts[1]] = parts[2]
            lines.append(",".join(parts) + "\n")
        tab = os.path.join(tempfile.gettempdir(), f"dtg_sustained_rank{rank}.csv")
        open(tab, "w").write("".join(lines))
        p = subprocess.run([sys.executable, "-u", os.path.abspath(__file__), "_time", "--table", tab,
                            "--seconds", str(a.seconds), "--only", a.only or ""],
                           capture_output=True, text=True, timeout=600)
        if p.returncode != 0:
            print(p.stdout[-2000:], p.stderr[-3000:], flush=True)
            raise SystemExit(f"rank {rank} child failed")
        for line in p.stdout.splitlines():
            if line.startswith("{"):
                r = json.loads(line)
                r["rank"] = rank
                r["solution"] = label.get(r["key"])
                r["committed"] = committed.get(("GemmTunableOp_BFloat16_TN", r["key"]))
                res.write(json.dumps(r) + "\n")
                res.flush()
                print(json.dumps(r), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("cmd", choices=["list", "time", "_tune", "_time"])
    ap.add_argument("--out")
    ap.add_argument("--cands")
    ap.add_argument("--table", default=TABLE)
    ap.add_argument("--top", type=int, default=4)
    ap.add_argument("--seconds", type=float, default=2.0)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    {"list": cmd_list, "time": cmd_time, "_tune": _tune, "_time": _time_child}[a.cmd](a)


if __name__ == "__main__":
    main()
