#!/usr/bin/env bash
# Round 6: is the xGMI TP path bitwise reproducible run to run (kernel vs copy-engine gathers)?
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r6_regather_diag}
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_tp_xgmi_gpu.py -k regather -v --timeout 200 --timeout-method thread \
    -p no:cacheprovider > "$O/pytest.log" 2>&1; rc=$?
grep -E "PASSED|FAILED|assert .*noise|AssertionError" "$O/pytest.log" | head -20
exit $rc
