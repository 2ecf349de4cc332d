#!/bin/bash
# colsum (RMSNorm weight-gradient column sums) on a 256-workgroup grid: norm tests, then the
# kernel's time in a profiled bench step (compare profiles/r3/s40: 65 launches, 1.17 ms).
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/r3_s44
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "norm" -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 3 --warmup 2 --fsdp-mem-steps 0 \
  > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
grep -h "^{" $O/prof.log | grep -oE '"ms_per_step": [0-9.]+'
