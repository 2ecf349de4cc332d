#!/usr/bin/env bash
# Attention kernel iteration: forward variants' numerics, then the same-process A/B.
#   gpurun -- bash gpujobs/r5_fa.sh <tag> "<variants>"
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r5_fa}
variants=${2:-v0,p64}
O=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "fwd_variants or d128_gqa or d64_mha" -x -q \
    --timeout 120 --timeout-method thread > "$O/pytest.log" 2>&1 || { tail -40 "$O/pytest.log"; exit 1; }
tail -2 "$O/pytest.log"
timeout -k 10 400 python -u tools/bench_attention.py --ab "$variants" > "$O/ab.jsonl" 2>&1 || { tail -20 "$O/ab.jsonl"; exit 1; }
cat "$O/ab.jsonl"
