#!/usr/bin/env bash
# Attention backward A/B: an environment knob of the dK/dV launch, same process, interleaved.
#   gpurun -- bash gpujobs/r5_fa_bwd.sh <tag> "VAR=v1,v2,..."
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r5_fa_bwd}
ab=${2:-DTG_FA_KV_SPLIT=1,2,3,4}
O=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 500 python -u tools/bench_attention.py --ab-bwd "$ab" --ab-tolerant > "$O/ab_bwd.jsonl" 2>&1 \
    || { tail -20 "$O/ab_bwd.jsonl"; exit 1; }
grep -v amdgpu.ids "$O/ab_bwd.jsonl"
