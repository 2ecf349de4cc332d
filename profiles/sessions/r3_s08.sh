#!/bin/bash
# swiglu_bwd_t tile shapes and adamw_ launch shapes: kernel tests, kernel bandwidth, bench A/B.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r3_s08
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "adamw or swiglu" -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python -u tools/bench_kernels.py > $O/kernels.log 2>&1 || { tail -20 $O/kernels.log; exit 1; }
grep kernel $O/kernels.log
for i in 1 2; do
  for tl in 64x64 64x128 128x128; do
    DTG_SWIGLU_TILE=$tl timeout -k 10 240 python -u bench.py --steps 10 --warmup 3 --fsdp-mem-steps 0 \
      > $O/bench_sg${tl}_$i.log 2>&1 || { tail -20 $O/bench_sg${tl}_$i.log; exit 1; }
    echo "swiglu tile=$tl run $i: $(tail -1 $O/bench_sg${tl}_$i.log | grep -oE '"ms_per_step": [0-9.]+')"
  done
done
