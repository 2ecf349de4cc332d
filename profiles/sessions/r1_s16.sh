#!/bin/bash
# TunableOp tuning of the TN backward GEMM shapes, merged into the table, then bench with it.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s16
export TMPDIR=/tmp
timeout -k 10 900 python -u tools/tune_gemms.py --which dx_tn,dw_tn --max-ms 25 --iters 10 --out gpurun_out/s16/tunableop_tn.csv > gpurun_out/s16/tune.log 2>&1
rc=$?; echo "tune rc=$rc"; tail -3 gpurun_out/s16/tune.log
[ $rc -eq 0 ] || exit $rc
cp tunableop/tunableop_results_partial.csv gpurun_out/s16/table_before.csv
python tools/merge_tunableop.py tunableop/tunableop_results_partial.csv gpurun_out/s16/tunableop_tn.csv
cp tunableop/tunableop_results_partial.csv gpurun_out/s16/table_merged.csv
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/s16/bench_tuned.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/s16/bench_tuned.log | cut -c1-300
exit $rc
