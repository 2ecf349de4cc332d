#!/bin/bash
# The committed table with the TP = 8 shapes merged: every pinned solution against f32.
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/r3_s36
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_tunableop_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
