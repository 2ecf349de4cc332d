#!/bin/bash
# Kernel-time profiles after the TN/fused-MLP change: Llama-3-8B bench and 405B (2 layers).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s18
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/s18/b8 -o run -- python3 bench.py --steps 3 --warmup 2 > gpurun_out/s18/b8.log 2>&1
rc=$?; echo "8b trace rc=$rc"; tail -1 gpurun_out/s18/b8.log | cut -c1-200
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/s18/b405 -o run -- python3 tools/bench_405b_depth.py --depths 2 --steps 2 --warmup 1 > gpurun_out/s18/b405.log 2>&1
rc=$?; echo "405 trace rc=$rc"; tail -1 gpurun_out/s18/b405.log | cut -c1-200
find gpurun_out/s18 -name "*.csv" -size +20M -delete
exit $rc
