#!/usr/bin/env bash
# r4_s36: Llama-3.1-405B as rank 0 of one 8-GPU node at depth 100 (host RSS ~250 GB by the
# per-layer fit of r4_s04, under the box's command limit), the deepest that fits with margin.
set -o pipefail
RING=auto bash tools/run_405b_node_w8.sh r4_s36 100
