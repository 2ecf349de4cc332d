#!/bin/bash
# Llama-3.1-405B launcher: one tmux session per host in ./hosts.
# MI355X sizing: pure-bf16 params+grads+AdamW = 8 B/param = 3.25 TB, i.e.
# 406 GB/GPU at 8 GPUs (does not fit 288 GB) and 203 GB/GPU at 16 GPUs (fits without offload).
# So: >= 2 nodes run with --cpu-offload off; a single node needs --cpu-offload on (host RAM).
set -euo pipefail
EXP=${1:-llama-405b}
HOSTS_FILE=${HOSTS_FILE:-hosts}
NNODES=$(grep -c '^' "$HOSTS_FILE")
OFFLOAD=$([ "$NNODES" -ge 2 ] && echo off || echo on)
HEAD=$(head -n 1 "$HOSTS_FILE")
CWD=$(pwd)
xargs -a "$HOSTS_FILE" -I{} ssh {} tmux new-session -d -s dtg405 -c "$CWD" \
  "env OMP_NUM_THREADS=26 HSA_ENABLE_IPC_MODE_LEGACY=0 TORCH_NCCL_AVOID_RECORD_STREAMS=1 \
   TORCHELASTIC_ERROR_FILE=../error.json \
   python -m torch.distributed.run --rdzv-id dtg405-$EXP --rdzv-backend c10d --rdzv-endpoint $HEAD:5001 \
   --nnodes $NNODES --nproc-per-node 8 --redirects 3 --log-dir ../logs \
   train_llm.py --experiment-name $EXP --dataset-name synthetic --model-name meta-llama/Llama-3.1-405B \
   --batch-size 1 --seq-length 4096 --cpu-offload $OFFLOAD --log-freq 1 ${INIT_FROM:+--init-from $INIT_FROM}"
