#!/bin/bash
# dQ kernel: software-pipelined tile body vs plain (same-process A/B, bitwise check) + tests + step.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r3_s09
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "flash or attention" -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u tools/bench_attention.py --ab-bwd plain,pipe > $O/ab_bwd.log 2>&1 || { tail -20 $O/ab_bwd.log; exit 1; }
grep case $O/ab_bwd.log
for i in 1 2; do
  for v in plain pipe; do
    DTG_FA_DQ=$v timeout -k 10 240 python -u bench.py --steps 10 --warmup 3 --fsdp-mem-steps 0 \
      > $O/bench_${v}_$i.log 2>&1 || { tail -20 $O/bench_${v}_$i.log; exit 1; }
    echo "dq=$v run $i: $(tail -1 $O/bench_${v}_$i.log | grep -oE '"ms_per_step": [0-9.]+')"
  done
done
