#!/bin/bash
# adamw_t_ tile widths: kernel test + kernel bandwidth + same-box bench A/B (W^T off / 64 / 128 /
# 256-column tiles), then the FSDP memory row at W = 4 (ranks sharing the GPU).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r3_s07
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "adamw" -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/pytest_adamw.log 2>&1 || { tail -30 $O/pytest_adamw.log; exit 1; }
tail -1 $O/pytest_adamw.log
timeout -k 10 300 python -u tools/bench_kernels.py --only adamw > $O/kernels_adamw.log 2>&1 || { tail -20 $O/kernels_adamw.log; exit 1; }
grep kernel $O/kernels_adamw.log
for i in 1 2; do
  for cfg in "1 64" "0 64" "1 128" "1 256"; do
    set -- $cfg
    DTG_WEIGHT_T=$1 DTG_ADAMT_TC=$2 timeout -k 10 240 python -u bench.py --steps 10 --warmup 3 --fsdp-mem-steps 0 \
      > $O/bench_wt$1_tc$2_$i.log 2>&1 || { tail -20 $O/bench_wt$1_tc$2_$i.log; exit 1; }
    echo "wt=$1 tc=$2 run $i: $(tail -1 $O/bench_wt$1_tc$2_$i.log | grep -oE '"ms_per_step": [0-9.]+')"
  done
done
W=4 LIMIT=600 bash tools/run_fsdp_mem_shared.sh r3_s07
