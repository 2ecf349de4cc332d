#!/bin/bash
# TP=2 Llama with xGMI TP collectives vs single device (2 ranks on one GPU).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s22
export TMPDIR=/tmp
timeout -k 10 240 python -u -m pytest tests/test_tp_xgmi_gpu.py tests/test_xgmi_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/s22/pytest.log 2>&1
rc=$?; echo "rc=$rc"; tail -25 gpurun_out/s22/pytest.log
exit $rc
