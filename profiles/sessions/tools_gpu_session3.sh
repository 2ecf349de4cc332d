#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --tunableop off > gpurun_out/bench_notune.log 2>&1
rc=$?; echo "bench(off) rc=$rc"; tail -1 gpurun_out/bench_notune.log | cut -c1-400
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python bench.py --steps 5 --warmup 3 --tunableop tune > gpurun_out/bench_tune.log 2>&1
rc=$?; echo "bench(tune) rc=$rc"; tail -1 gpurun_out/bench_tune.log | cut -c1-400
[ $rc -ne 0 ] && exit $rc
mkdir -p gpurun_out/tunableop && cp tunableop/*.csv gpurun_out/tunableop/ 2>/dev/null
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --tunableop use > gpurun_out/bench_use.log 2>&1
rc=$?; echo "bench(use) rc=$rc"; tail -1 gpurun_out/bench_use.log | cut -c1-400
exit $rc
