#!/bin/bash
# Transpose tile 64 vs 128 (kernel roofline), transpose numerics, bench with the new default.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s34
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "transpose or linear_bwd or mlp" > gpurun_out/s34/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/s34/pytest.log
[ $rc -eq 0 ] || exit $rc
for t in 64 128; do
  DTG_TRANSPOSE_TILE=$t timeout -k 10 200 python -u tools/bench_kernels.py > gpurun_out/s34/kernels_t$t.jsonl 2>&1
  rc=$?; echo "tile $t rc=$rc"; grep transpose gpurun_out/s34/kernels_t$t.jsonl
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/s34/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/s34/bench.log | cut -c1-200
exit $rc
