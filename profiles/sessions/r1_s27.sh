#!/bin/bash
# AdamW 2-vector unroll + RMSNorm bwd row pipelining: kernel tests, bench, short kernel profile.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s27
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "adamw or rmsnorm" > gpurun_out/s27/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/s27/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/s27/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/s27/bench.log | cut -c1-200
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/s27/prof -o run -- python3 bench.py --steps 3 --warmup 2 > gpurun_out/s27/prof.log 2>&1
rc=$?; echo "prof rc=$rc"
exit $rc
