#!/usr/bin/env bash
# r4_s04: attention dropout in the flash kernels + host gradient ring (GPU tests), then 405B W = 8
# rank 0 with the ring at depths 8 and 80.
set -o pipefail
out=gpurun_out/r4_s04
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_kernels_gpu.py -k "attn or attention or gpt2 or dropout" > "$out/pytest_attn.log" 2>&1 \
    || { tail -40 "$out/pytest_attn.log"; exit 1; }
tail -1 "$out/pytest_attn.log"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
    tests/test_engines_rccl_gpu.py -k "offload" > "$out/pytest_ring.log" 2>&1 || { tail -30 "$out/pytest_ring.log"; exit 1; }
tail -1 "$out/pytest_ring.log"
RING=auto bash tools/run_405b_node_w8.sh r4_s04 8 80
