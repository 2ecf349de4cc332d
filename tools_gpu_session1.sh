#!/bin/bash
# GPU session: kernel numerics tests, flagship bench, rocprofv3 kernel stats.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: pytest crashed"; exit $rc; fi
timeout -k 10 600 python bench.py --steps 5 --warmup 2 > gpurun_out/bench1.log 2>&1
rc=$?
echo "bench rc=$rc"; tail -3 gpurun_out/bench1.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof1 -o run -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/prof1.log 2>&1
rc=$?
echo "rocprof rc=$rc"; tail -3 gpurun_out/prof1.log
exit $rc
