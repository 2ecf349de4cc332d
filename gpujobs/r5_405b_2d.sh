#!/usr/bin/env bash
# Llama-3.1-405B on ONE 8-GPU node through chapter 07 (2-D: FSDP over dp x TP over tp) with
# chapter 05's CPU offload, measured as rank 0 of the W = 8 job (DTG_FAKE_WORLD=8: the other 7
# ranks are a fake process group -- the rank's shards, offload traffic, host AdamW and compute are
# the real job's; the TP / FSDP collectives are not).  Exact width and FULL depth (126 layers),
# seq 4096, activation checkpointing, parameters resident in HBM, host gradient ring.
# Usage: gpurun --timeout 1200 -- bash gpujobs/r5_405b_2d.sh <tag> "<tp>:<batch>[:depth] ..."
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r5_405b_2d}
runs=${2:-"8:8 4:4"}
O=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p $O
export TMPDIR=/tmp
( while true; do echo "[405b_2d] alive $(date +%T) $(grep MemAvailable /proc/meminfo)"; sleep 30; done ) & HB=$!
trap 'kill $HB; rm -rf /tmp/dtg405_2d' EXIT
grep -E "MemTotal|MemAvailable" /proc/meminfo > $O/meminfo_start.txt
SHARE=16
for spec in $runs; do
  IFS=: read tp b depth <<< "$spec"
  depth=${depth:-126}
  rm -rf /tmp/dtg405_2d
  log=$O/ch07_405b_tp${tp}_b${b}_d${depth}.log
  (cd 07-2d-parallel && DTG_FAKE_WORLD=8 OMP_NUM_THREADS=$SHARE timeout -k 10 560 python -u train_llm.py \
     -e r405_2d -m meta-llama/Llama-3.1-405B --num-layers $depth -b $b -s 4096 -d synthetic --num-workers 1 \
     --tp $tp --save-dir /tmp/dtg405_2d --ckpt-freq 100000 --max-steps 4 --log-freq 1 --cpu-offload on \
     --offload-params off --activation-checkpointing on --pin-numa on --cpu-share $SHARE ${EXTRA:-} > $log 2>&1)
  rc=$?
  echo "tp=$tp b=$b depth=$depth rc=$rc"
  grep -E "global_step': [34]," $log | grep -oE "'(tok/s|time/forward|time/backward|time/update|time/total|peak_alloc_gb|peak_reserved_gb|offload/[a-z0-9_]+|host/[a-z_]+)': [0-9.]+" | tr '\n' ' '; echo
  [ $rc -eq 0 ] || { tail -30 $log; exit $rc; }
done
