#!/bin/bash
# Multi-node launcher without a scheduler: one detached tmux session per host in
# `hosts`, each running torchrun with c10d rendezvous on the first host.
#   ./launch_ssh_tmux.sh <experiment-name> [chapter-dir] [extra train_llm.py args...]
# Stop:    xargs -a hosts -I{} ssh {} tmux kill-session -t dtg
# Monitor: find ../logs -name \*stderr.log | xargs tail -f     (or: python ../tools/top_cluster.py)
set -euo pipefail
EXP=${1:?experiment name}; shift
CHAPTER=${1:-02-distributed-data-parallel}; shift || true
HOSTS_FILE=${HOSTS_FILE:-hosts}
HEAD=$(head -n 1 "$HOSTS_FILE")
NNODES=$(grep -c '^' "$HOSTS_FILE")
CWD=$(pwd)
xargs -a "$HOSTS_FILE" -I{} ssh {} tmux new-session -d -s dtg -c "$CWD" \
  "env OMP_NUM_THREADS=1 HSA_ENABLE_IPC_MODE_LEGACY=0 TORCHELASTIC_ERROR_FILE=../error.json \
   python -m torch.distributed.run --rdzv-id dtg-$EXP --rdzv-backend c10d --rdzv-endpoint $HEAD:5001 \
   --nnodes $NNODES --nproc-per-node gpu --redirects 3 --log-dir ../logs \
   ../$CHAPTER/train_llm.py --experiment-name $EXP $*"
