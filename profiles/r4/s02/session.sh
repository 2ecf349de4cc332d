#!/usr/bin/env bash
# r4_s02: exact-size pinned offload buffers + Llama-3.1-405B as rank 0 of ONE 8-GPU node (W = 8).
set -o pipefail
out=gpurun_out/r4_s02
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
    tests/test_pinned_gpu.py > "$out/pytest.log" 2>&1 || { tail -30 "$out/pytest.log"; exit 1; }
tail -1 "$out/pytest.log"
bash tools/run_405b_node_w8.sh r4_s02 8 56
