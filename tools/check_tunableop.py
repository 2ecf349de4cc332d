#!/usr/bin/env python3
"""Numerics check of every solution in the committed TunableOp table (tunableop/).

TunableOp does not compare a candidate's output with the default kernel's unless
PYTORCH_TUNABLEOP_NUMERICAL_CHECK is set, so a tuned table can pin a solution that is fast and
wrong for its shape.  For every row this rebuilds the operands the key describes, runs the GEMM
once through the table (TunableOp on, tuning off) and once with TunableOp off (library default),
and compares both with an f32 product of the same bf16 operands.

    python tools/check_tunableop.py [--table PATH] [--out results.jsonl]

Key grammar (column-major BLAS, as PyTorch issues it for row-major tensors): for
`<ta><tb>_m_n_k[_B_batch]_ld_lda_ldb_ldc` the row-major product is C[n, m] = X[n, k] @ Y[k, m]
with Y = W.t() (W contiguous [m, k]) when ta == 't' else contiguous [k, m], and X contiguous
[n, k] when tb == 'n' else Z.t() (Z contiguous [k, n]).  GemmAndBias adds a bias[m] (F.linear);
GemmStridedBatched applies the same per batch (torch.bmm).
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def parse_key(key):
    parts = key.split("_")
    ta, tb = parts[0][0], parts[0][1]
    m, n, k = int(parts[1]), int(parts[2]), int(parts[3])
    batch = int(parts[5]) if parts[4] == "B" else None
    return ta, tb, m, n, k, batch


def operands(ta, tb, m, n, k, batch, dev, g):
    bshape = () if batch is None else (batch,)

    def rnd(*shape):
        return torch.randn(*bshape, *shape, device=dev, generator=g).bfloat16()

    y = rnd(m, k).transpose(-1, -2) if ta == "t" else rnd(k, m)
    x = rnd(n, k) if tb == "n" else rnd(k, n).transpose(-1, -2)
    return x, y


def run(op, x, y, bias):
    if op.startswith("GemmAndBias"):
        return torch.nn.functional.linear(x, y.transpose(-1, -2), bias)
    if op.startswith("GemmStridedBatched"):
        return torch.bmm(x, y)
    return torch.mm(x, y)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--table", default=os.path.join(ROOT, "tunableop", "tunableop_results_partial.csv"))
    ap.add_argument("--out", default=None)
    ap.add_argument("--tol", type=float, default=3e-2, help="max |err| / max |ref| counted as a failure")
    a = ap.parse_args()
    from dtg.utils.gemm_tuning import enable_tunableop

    dev = torch.device("cuda:0")
    enable_tunableop(tune=False, table=a.table)
    t = torch.cuda.tunable
    rows = []
    with open(a.table) as fp:
        for line in fp:
            f = line.strip().split(",")
            if len(f) >= 3 and not f[0].startswith("Validator"):
                rows.append((f[0], f[1], f[2]))
    out = open(a.out, "w") if a.out else None
    bad = 0
    g = torch.Generator(device=dev).manual_seed(0)
    for op, key, sol in rows:
        ta, tb, m, n, k, batch = parse_key(key)
        x, y = operands(ta, tb, m, n, k, batch, dev, g)
        bias = torch.randn(m, device=dev, generator=g).bfloat16() if op.startswith("GemmAndBias") else None
        ref = torch.matmul(x.float(), y.float())
        if bias is not None:
            ref = ref + bias.float()
        scale = ref.abs().max().item() + 1e-6
        t.enable(True)
        tuned = run(op, x, y, bias)
        t.enable(False)
        default = run(op, x, y, bias)
        torch.cuda.synchronize()
        rec = {"op": op, "key": key, "solution": sol,
               "tuned_err": (tuned.float() - ref).abs().max().item() / scale,
               "default_err": (default.float() - ref).abs().max().item() / scale,
               "tuned_finite": bool(torch.isfinite(tuned).all().item())}
        rec["ok"] = rec["tuned_finite"] and rec["tuned_err"] <= a.tol
        bad += not rec["ok"]
        line = json.dumps(rec)
        print(line, flush=True)
        if out:
            out.write(line + "\n")
        del x, y, ref, tuned, default
    print(json.dumps({"rows": len(rows), "failed": bad}), flush=True)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
