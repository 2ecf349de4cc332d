#!/bin/bash
# dK/dV with 64-query items (two-half software pipeline): GPU tests, kernel A/B across the
# attention shapes, then the full 8B step with DTG_FA_KV_QB=32 vs 64 alternating.
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/r3_s39
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "flash or attention" -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python -u tools/bench_attention.py --ab-bwd DTG_FA_KV_QB=32,64 --ab-tolerant > $O/ab_bwd.log 2>&1 || { tail -20 $O/ab_bwd.log; exit 1; }
grep case $O/ab_bwd.log
for v in 32 64 32 64; do
  DTG_FA_KV_QB=$v timeout -k 10 240 python -u bench.py --steps 10 --warmup 3 --fsdp-mem-steps 0 > $O/bench_qb$v.log 2>&1 \
    || { tail -20 $O/bench_qb$v.log; exit 1; }
  echo "qb=$v: $(tail -1 $O/bench_qb$v.log | grep -oE '"ms_per_step": [0-9.]+')"
done
