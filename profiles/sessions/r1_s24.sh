#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s24
export TMPDIR=/tmp
timeout -k 10 300 python tools/bench_gemm_square.py > gpurun_out/s24/gemm_square.jsonl 2>&1
rc=$?; echo "rc=$rc"; cat gpurun_out/s24/gemm_square.jsonl
exit $rc
