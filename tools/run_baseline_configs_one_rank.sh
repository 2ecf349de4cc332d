#!/bin/bash
# BASELINE configs 02 / 04 / 06 / 07 at 8 GPUs, measured as ONE rank of the 8-rank job on one
# MI355X (DTG_FAKE_WORLD=8: the other ranks are a fake process group, so these are per-rank
# compute + memory WITHOUT communication -- upper bounds for tok/s, exact for memory).
# Usage: gpurun --timeout 1200 -- bash tools/run_baseline_configs_one_rank.sh <tag>
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-baseline_one_rank}
mkdir -p $O
export TMPDIR=/tmp
( while true; do echo "[one_rank] alive $(date +%T)"; sleep 30; done ) & HB=$!
trap 'kill $HB; rm -rf /tmp/dtg_or' EXIT
COMMON="-d synthetic --num-workers 1 --save-dir /tmp/dtg_or --ckpt-freq 100000 --max-steps 8 --log-freq 2"
run() {  # name dir args...
  local name=$1 dir=$2; shift 2
  rm -rf /tmp/dtg_or
  (cd $dir && DTG_FAKE_WORLD=8 timeout -k 10 400 python -u train_llm.py -e $name "$@" $COMMON > $O/$name.log 2>&1)
  local rc=$?
  echo "$name rc=$rc: $(grep -E "global_step': 8," $O/$name.log | grep -oE "'(tok/s|tok/s/gpu|peak_alloc_gb|peak_alloc_in_gb|time/forward|time/backward|time/update)': [0-9.]+" | tr '\n' ' ')"
  [ $rc -eq 0 ] || { tail -30 $O/$name.log; exit $rc; }
}
run ch02_ddp_w8 02-distributed-data-parallel -m meta-llama/Meta-Llama-3-8B -b 16
run ch04_fsdp_w8 04-fully-sharded-data-parallel -m meta-llama/Meta-Llama-3-8B -b 16
run ch06_tp8 06-tensor-parallel -m meta-llama/Llama-3.1-8B -b 16
run ch07_tp4dp2 07-2d-parallel -m meta-llama/Llama-3.1-8B -b 16 --tp 4
