#!/usr/bin/env bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
for e in kernel dma; do
  DTG_SHARED_DEVICE=1 timeout -k 10 120 python -u -m torch.distributed.run --nnodes 1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port $((29600 + RANDOM % 300)) tools/diag_regather.py --engine $e 2>&1 | grep -E "^\{|Error" || exit 1
done
