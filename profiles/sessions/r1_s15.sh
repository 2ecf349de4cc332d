#!/bin/bash
# TN backward layouts: transpose kernel numerics + bandwidth, bench.py under each DTG_LINEAR_BWD mode.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s15
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s15/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/s15/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_gemm_layouts.py > gpurun_out/s15/gemm_layouts.jsonl 2>&1
rc=$?; echo "layouts rc=$rc"
[ $rc -eq 0 ] || exit $rc
for m in native auto tn; do
  DTG_LINEAR_BWD=$m timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/s15/bench_$m.log 2>&1
  rc=$?; echo "bench $m rc=$rc"; tail -1 gpurun_out/s15/bench_$m.log | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
done
exit 0
