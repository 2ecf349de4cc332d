#!/usr/bin/env bash
# Rank 0 of the dp8 ZeRO bench alone (DTG_FAKE_WORLD=8: the other ranks are a fake process group,
# so this is the per-rank compute of the N = 8 step, no communication) next to the N = 1 bench,
# same box, at the final HEAD.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r6_fake8}
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py > "$O/bench_n1.log" 2>&1 || { tail -20 "$O/bench_n1.log"; exit 1; }
tail -1 "$O/bench_n1.log" | cut -c1-300
DTG_FAKE_WORLD=8 timeout -k 10 300 python -u bench.py --gpus 8 --fsdp-mem-steps 0 > "$O/bench_fake8.log" 2>&1 \
    || { tail -20 "$O/bench_fake8.log"; exit 1; }
tail -1 "$O/bench_fake8.log" | cut -c1-400
