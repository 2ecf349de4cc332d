#!/usr/bin/env bash
# r4_s26: pinned buffers tied to their memory + the offload engines that use them; chapter 05 with
# the measured --offload-grad-ring auto policy (resident: ring on; params on host: ring off).
set -o pipefail
out=gpurun_out/r4_s26
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
    tests/test_pinned_gpu.py tests/test_engines_rccl_gpu.py tests/test_dw_gemm_gpu.py > "$out/pytest.log" 2>&1 \
    || { tail -40 "$out/pytest.log"; exit 1; }
tail -1 "$out/pytest.log"
timeout -k 10 600 bash tools/run_chapters_gpu.sh r4_s26 ch05 || exit 1
