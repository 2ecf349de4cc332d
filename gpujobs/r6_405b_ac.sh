#!/usr/bin/env bash
# Round 6: the ch07 tp 4 x dp 2 + offload 405B one-node recipe as rank 0 of W = 8
# (DTG_FAKE_WORLD=8), exact width, depth 100, b4 x 4096, finite data -- with every layer
# checkpointed (the reference) against `--ac-layers` budgets.  auto plans against
# --ac-budget-gb ${BUDGET:-256}: 280 GB minus what 26 more layers add at 126 layers (0.80 GB
# parameter shard + 0.13 GB checkpointed input each, ~24 GB), so the projected 126-layer peak stays
# <= 280 GB of the 309 GB (288 GiB) HBM.
# Usage: gpurun --timeout 1200 -- bash gpujobs/r6_405b_ac.sh <tag> "all auto auto+rg 40"
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r6_405b_ac}
runs=${2:-"all auto"}
O=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p $O
export TMPDIR=/tmp
( while true; do echo "[405b_ac] alive $(date +%T) $(grep MemAvailable /proc/meminfo)"; sleep 30; done ) & HB=$!
trap 'kill $HB; rm -rf /tmp/dtg405_ac' EXIT
SHARE=16
for spec in $runs; do
  IFS=+ read ac rg <<< "$spec"   # e.g. "auto+rg": --ac-layers auto --sp-regather on
  extra=""; [ "$rg" = rg ] && extra="--sp-regather on"
  rm -rf /tmp/dtg405_ac
  log=$O/ch07_405b_tp${TP:-4}_b${TP:-4}_d100_ac_${spec}.log
  (cd 07-2d-parallel && DTG_FAKE_WORLD=8 OMP_NUM_THREADS=$SHARE timeout -k 10 480 python -u train_llm.py \
     -e r405_ac -m meta-llama/Llama-3.1-405B --num-layers 100 -b ${TP:-4} -s 4096 -d synthetic --num-workers 1 \
     --tp ${TP:-4} --save-dir /tmp/dtg405_ac --ckpt-freq 100000 --max-steps ${STEPS:-6} --log-freq 1 --cpu-offload on \
     --offload-params off --activation-checkpointing on --ac-layers $ac --ac-budget-gb ${BUDGET:-256} \
     --pin-numa on --cpu-share $SHARE $extra > $log 2>&1)
  rc=$?
  echo "$spec rc=$rc"
  grep -E "ac-layers auto|activation checkpointing:" $log
  grep -E "global_step': [3-9]," $log | grep -oE "'(running_loss|time/forward|time/backward|time/total|peak_alloc_gb|peak_resv_gb|ac/layers)': [0-9.]+" | tr '\n' ' '; echo
  [ $rc -eq 0 ] || { tail -30 $log; exit $rc; }
done
