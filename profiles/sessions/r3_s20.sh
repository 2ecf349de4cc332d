#!/bin/bash
# dK/dV kernel at one vs two waves per SIMD (DTG_FA_KV_OCC): tests, in-process A/B, bench step.
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/r3_s20
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "flash" -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u tools/bench_attention.py --ab-bwd DTG_FA_KV_OCC=1,2 > $O/ab_bwd.log 2>&1 || { tail -20 $O/ab_bwd.log; exit 1; }
grep case $O/ab_bwd.log
for i in 1 2; do
  for v in 1 2; do
    DTG_FA_KV_OCC=$v timeout -k 10 240 python -u bench.py --steps 10 --warmup 3 --fsdp-mem-steps 0 > $O/bench_occ${v}_$i.log 2>&1 \
      || { tail -20 $O/bench_occ${v}_$i.log; exit 1; }
    echo "kv_occ=$v run $i: $(tail -1 $O/bench_occ${v}_$i.log | grep -oE '"ms_per_step": [0-9.]+')"
  done
done
