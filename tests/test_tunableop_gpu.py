"""Every solution pinned in the committed TunableOp table computes the right product.

TunableOp ranks candidates on time; one pinned hipBLASLt solution for GPT-2's batched
attention-score GEMM returned values of order 1e33 and turned chapter 01's loss into NaN
(profiles/r2/s35/).  tools/check_tunableop.py rebuilds each row's operands and compares the
table's kernel with an f32 product.  It runs in a child process so that enabling TunableOp does
not change the GEMM solutions of the other tests in this session.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def test_table_keys_parse():
    from check_tunableop import parse_key

    rows = [l.split(",") for l in open(os.path.join(ROOT, "tunableop", "tunableop_results_partial.csv"))
            if l.startswith("Gemm")]
    assert rows
    for op, key, *_ in rows:
        ta, tb, m, n, k, batch = parse_key(key)
        assert ta in "nt" and tb in "nt" and min(m, n, k) > 0
        assert (batch is not None) == op.startswith("GemmStridedBatched"), key


@pytest.mark.gpu
def test_tuned_solutions_match_f32(cuda):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "check_tunableop.py")], capture_output=True,
                       text=True, timeout=300, cwd=ROOT)
    bad = [l for l in r.stdout.splitlines() if '"ok": false' in l]
    assert r.returncode == 0 and not bad, (r.stdout[-3000:], r.stderr[-2000:])
