#!/usr/bin/env bash
# Register-blocked transpose (DTG_TRANSPOSE_TILE=reg) vs the LDS-tiled kernels: numerics, then
# the transpose cases of tools/bench_kernels.py (8B shapes, A B A B order).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5_transpose}
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -k "transpose or swiglu or adamw_t" -x -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider > "$O/pytest.log" 2>&1 || { tail -30 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
timeout -k 10 300 python -u tools/bench_kernels.py --only transpose,swiglu_bwd_t,adamw_t_ > "$O/bench.log" 2>&1 || { tail -20 "$O/bench.log"; exit 1; }
grep -v amdgpu.ids "$O/bench.log"
