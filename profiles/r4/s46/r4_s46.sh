#!/usr/bin/env bash
# r4_s46: the kernel, engine and model GPU tests with the fused RoPE backward switched on.
set -o pipefail
out=gpurun_out/r4_s46
mkdir -p "$out"
export TMPDIR=/tmp
DTG_FA_ROPE_FUSED=1 timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_kernels_gpu.py tests/test_fa_rope_fused_gpu.py tests/test_engines_gpu.py tests/test_graph_gpu.py \
    > "$out/pytest_fused_on.log" 2>&1 || { tail -40 "$out/pytest_fused_on.log"; exit 1; }
tail -1 "$out/pytest_fused_on.log"
