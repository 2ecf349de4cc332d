#!/usr/bin/env bash
# Tune the 405B tp 4 x dp 2 recipe's 13 GEMM shapes (recorded by r5_tune_405b.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5_tune_tp4}
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 1100 python -u tools/tune_gemms.py tunableop/untuned/untuned_405b_tp4.csv --out $O/tuned_tp4.csv \
    --budget-s 960 --shape-timeout-s 150 > $O/tune.log 2>&1; rc=$?
grep "done\|tuned " $O/tune.log | tail -20
exit $rc
