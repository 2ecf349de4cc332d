#!/bin/bash
# Pair-read transposed store phase (transpose2d, swiglu_bwd_t): GPU tests, kernel A/B at the
# 8B step shapes, then the bench with the pair forms on (env) vs off, same box.
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/r3_s31
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "transpose2d or swiglu_bwd_t" -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u tools/bench_kernels.py --only swiglu_bwd_t,transpose > $O/kernels.log 2>&1 || { tail -20 $O/kernels.log; exit 1; }
cat $O/kernels.log | grep kernel
for v in 0 1 0 1; do
  DTG_TRANSPOSE_PAIR=$v DTG_SWIGLU_PAIR=$v timeout -k 10 240 python -u bench.py --steps 10 --warmup 3 --fsdp-mem-steps 0 > $O/bench_pair$v.log 2>&1 \
    || { tail -20 $O/bench_pair$v.log; exit 1; }
  echo "pair=$v: $(tail -1 $O/bench_pair$v.log | grep -oE '"ms_per_step": [0-9.]+')"
done
