#!/bin/bash
# Fused SwiGLU-MLP node (transposing backward) + tuned TN table: GPU tests, bench, 405B depth bench.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s17
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s17/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/s17/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/s17/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/s17/bench.log | cut -c1-400
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/bench_405b_depth.py --depths 2,4 --steps 3 --warmup 2 > gpurun_out/s17/bench_405b.log 2>&1
rc=$?; echo "405b rc=$rc"; tail -3 gpurun_out/s17/bench_405b.log
exit $rc
