#!/bin/bash
# Full GPU suite after the graph/GPT-2 changes; 405B depth bench with the optimizer timed separately.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s31
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s31/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/s31/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/bench_405b_depth.py --depths 2,4 --steps 3 --warmup 2 > gpurun_out/s31/bench_405b.log 2>&1
rc=$?; echo "405b rc=$rc"; grep -v amdgpu gpurun_out/s31/bench_405b.log | grep '{' | cut -c1-500
exit $rc
