#!/usr/bin/env bash
# r4_s12: dW GEMM variant 3 (ping-pong) numerics + microbench; the dW side-stream race test and
# same-box A/B (DTG_DW_STREAM).
set -o pipefail
out=gpurun_out/r4_s12
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
    tests/test_dw_gemm_gpu.py > "$out/pytest_dwg.log" 2>&1 || { tail -40 "$out/pytest_dwg.log"; exit 1; }
tail -1 "$out/pytest_dwg.log"
timeout -k 10 300 python -u tools/bench_dw_gemm.py > "$out/bench_dwg.jsonl" 2> "$out/bench_dwg.err" \
    || { tail -20 "$out/bench_dwg.err"; exit 1; }
cat "$out/bench_dwg.jsonl"
