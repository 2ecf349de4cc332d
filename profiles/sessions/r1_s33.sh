#!/bin/bash
# Memory-bound kernel roofline (timed) + PMC byte counts (two single-block passes).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s33
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/bench_kernels.py > gpurun_out/s33/kernels.jsonl 2>&1
rc=$?; echo "timed rc=$rc"; grep '{' gpurun_out/s33/kernels.jsonl
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/s33/fetch -o run -- python3 tools/bench_kernels.py > gpurun_out/s33/fetch.log 2>&1
rc=$?; echo "fetch rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/s33/write -o run -- python3 tools/bench_kernels.py > gpurun_out/s33/write.log 2>&1
rc=$?; echo "write rc=$rc"
exit $rc
