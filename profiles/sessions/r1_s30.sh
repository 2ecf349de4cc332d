#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s30
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_graph_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/s30/pytest.log 2>&1
rc=$?; echo "rc=$rc"; tail -8 gpurun_out/s30/pytest.log
exit $rc
