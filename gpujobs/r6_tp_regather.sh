#!/usr/bin/env bash
# Round 6: TP GPU tests (xGMI transports, incl. --sp-regather bitwise), then the 405B tp 4 rank at
# depth 100 with every layer checkpointed, --ac-layers auto, and auto + --sp-regather.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r6_tp_regather}
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_tp_xgmi_gpu.py tests/test_transport_auto_gpu.py -x -q --timeout 200 \
    --timeout-method thread -p no:cacheprovider > "$O/pytest.log" 2>&1 || { tail -30 "$O/pytest.log"; exit 1; }
tail -n 1 "$O/pytest.log"
bash gpujobs/r6_405b_ac.sh ${1:-r6_tp_regather} "${2:-all auto auto+rg}"
