#!/usr/bin/env bash
# Round 6: the iterative --ac-layers auto planner (re-checks the peak after steps 3 and 4) on
# chapter 05's FSDP W = 8 rank and chapter 07's tp 4 x dp 2 rank with --sp-regather, depth 100,
# budget 256 GB; 7 steps each, the last two reported.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r6_405b_ac_iter}
STEPS=7 EXTRA="--ac-layers auto --ac-budget-gb 256" bash tools/run_405b_node_w8.sh ${tag}_ch05 100 || exit 1
grep -h "ac-layers auto" gpurun_out/${tag}_ch05/*.log | cut -c1-260
STEPS=7 bash gpujobs/r6_405b_ac.sh ${tag}_ch07 "auto+rg" || exit 1
