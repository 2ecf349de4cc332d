#!/usr/bin/env bash
# Kernel breakdown of the recommended 405B one-node recipe (ch07 tp 4 x dp 2 + CPU offload, rank 0
# of W = 8, exact width): depth 20, 3 steps under rocprofv3 --kernel-trace --stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5_405b_tp4_prof}
mkdir -p "$O"
export TMPDIR=/tmp
( while true; do sleep 45; echo "[prof] alive"; done ) & HB=$!
trap 'kill $HB 2>/dev/null; rm -rf /tmp/tp4prof' EXIT
cd 07-2d-parallel || exit 1
DTG_FAKE_WORLD=8 OMP_NUM_THREADS=16 timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$O/trace" -o run \
    --output-format csv -- python3 -u train_llm.py -e prof -m meta-llama/Llama-3.1-405B --num-layers 20 -b 4 -s 4096 \
    -d synthetic --num-workers 1 --tp 4 --save-dir /tmp/tp4prof --ckpt-freq 100000 --max-steps 3 --log-freq 1 \
    --cpu-offload on --offload-params off --activation-checkpointing on --pin-numa on --cpu-share 16 \
    > "$O/run.log" 2>&1 || { tail -20 "$O/run.log"; exit 1; }
grep -oE "'global_step': [0-9]+|'time/total': [0-9.]+|'running_loss': [0-9.]+" "$O/run.log" | paste -sd' '
head -15 "$O/trace/run_kernel_stats.csv" | cut -c1-150
