#!/bin/bash
# Split attention backward: numerics (both occupancies), kernel timings, end-to-end bench.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for occ in 1 2; do
  DTG_FA_OCC=$occ timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -x -k attn > gpurun_out/s7_pytest_occ$occ.log 2>&1
  rc=$?; echo "pytest attn occ=$occ rc=$rc"; tail -2 gpurun_out/s7_pytest_occ$occ.log
  [ $rc -ne 0 ] && exit $rc
done
for shape in llama8b rime gpt2; do
  for cfg in "DTG_FA_OCC=1" "DTG_FA_OCC=2" "DTG_FA_BWD=1"; do
    env $cfg timeout -k 10 120 python tools/bench_attention.py --shape $shape >> gpurun_out/s7_attn.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "attn bench $shape $cfg rc=$rc"; tail -3 gpurun_out/s7_attn.log; exit $rc; }
  done
done
grep shape gpurun_out/s7_attn.log
timeout -k 10 400 python bench.py --steps 6 --warmup 2 > gpurun_out/s7_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/s7_bench.log | cut -c1-400
exit $rc
