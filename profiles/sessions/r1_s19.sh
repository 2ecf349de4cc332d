#!/bin/bash
# TN loss-head GEMMs (even 4096-row chunks): tune the new shapes, merge, GPU tests, bench.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s19
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s19/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/s19/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/tune_gemms.py --only lm_head --tokens 4096 --which fwd,dx_tn,dw_tn --max-ms 25 --iters 10 --out gpurun_out/s19/tunableop_head.csv > gpurun_out/s19/tune.log 2>&1
rc=$?; echo "tune rc=$rc"; tail -2 gpurun_out/s19/tune.log
[ $rc -eq 0 ] || exit $rc
python tools/merge_tunableop.py tunableop/tunableop_results_partial.csv gpurun_out/s19/tunableop_head.csv
cp tunableop/tunableop_results_partial.csv gpurun_out/s19/table_merged.csv
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/s19/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/s19/bench.log | cut -c1-300
exit $rc
