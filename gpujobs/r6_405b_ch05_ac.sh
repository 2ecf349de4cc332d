#!/usr/bin/env bash
# Round 6: chapter 05's 405B recipe (FSDP W = 8 + offload, rank 0 via DTG_FAKE_WORLD=8, depth 100)
# with every layer checkpointed vs --ac-layers auto (budget 256 GB = 280 minus what 26 more layers
# add at full depth).  Same box.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r6_405b_ch05_ac}
bash tools/run_405b_node_w8.sh ${tag}_all 100 || exit 1
EXTRA="--ac-layers auto --ac-budget-gb 256" bash tools/run_405b_node_w8.sh ${tag}_auto 100 || exit 1
grep -h "ac-layers auto" gpurun_out/${tag}_auto/*.log
