#!/bin/bash
# Batch-size sweep of the flagship bench (288 GB HBM), full GPU test suite, 405B depth bench.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s23
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/s23/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/s23/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
for b in 16 24 32; do
  timeout -k 10 400 python bench.py --steps 8 --warmup 3 --batch-size $b > gpurun_out/s23/bench_b$b.log 2>&1
  rc=$?; echo "bench b=$b rc=$rc"; tail -1 gpurun_out/s23/bench_b$b.log | cut -c1-200; grep -o '"peak_mem_gb[^,]*' gpurun_out/s23/bench_b$b.log
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 600 python -u tools/bench_405b_depth.py --depths 2,4 --steps 3 --warmup 2 > gpurun_out/s23/bench_405b.log 2>&1
rc=$?; echo "405b rc=$rc"; tail -3 gpurun_out/s23/bench_405b.log | cut -c1-400
exit $rc
