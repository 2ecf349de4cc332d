#!/bin/bash
# xGMI direct-peer collectives: 2 processes on one GPU (protocol + arithmetic).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s21
export TMPDIR=/tmp
timeout -k 10 180 python -u -m pytest tests/test_xgmi_gpu.py -x -v --timeout 150 --timeout-method thread > gpurun_out/s21/pytest_xgmi.log 2>&1
rc=$?; echo "xgmi rc=$rc"; tail -15 gpurun_out/s21/pytest_xgmi.log
exit $rc
