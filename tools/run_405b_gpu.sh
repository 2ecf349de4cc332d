#!/bin/bash
# Chapter 05's engine at the exact Llama-3.1-405B width (hidden 16,384, FFN 53,248, 128/8 heads,
# vocab 128,256) and reduced depth (--num-layers 2 and 4) on one MI355X: FSDP transformer wrap,
# activation checkpointing, b1 x 4096, with and without CPU offload.  Logs feed
# tools/extrapolate_405b.py (per-layer = (d4 - d2) / 2).
# Usage: gpurun --timeout 1200 -- bash tools/run_405b_gpu.sh <tag>
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r405}
mkdir -p "$OUT"
export TMPDIR=/tmp
TR="python -u -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29573"
COMMON="-m meta-llama/Llama-3.1-405B -b 1 -s 4096 -d synthetic --save-dir /tmp/dtg405 --ckpt-freq 100000 --num-workers 1 --max-steps ${STEPS:-6} --log-freq 1"
( while sleep 30; do echo "[405b] alive $(date +%T)"; done ) &
HB=$!
trap "kill $HB; rm -rf /tmp/dtg405" EXIT
run() {  # name, extra args...
  local name=$1; shift
  rm -rf /tmp/dtg405
  (cd 05-training-llama-405b && timeout -k 10 ${LIMIT:-420} $TR train_llm.py -e $name $COMMON "$@" > "$OUT/$name.log" 2>&1)
  local rc=$?
  echo "$name rc=$rc"; grep -E "global_step" "$OUT/$name.log" | tail -1 | cut -c1-400
  [ $rc -ne 0 ] && tail -30 "$OUT/$name.log"
  return $rc
}
run ch05_405b_d2_no_offload --num-layers 2 --cpu-offload off && \
run ch05_405b_d4_no_offload --num-layers 4 --cpu-offload off && \
run ch05_405b_d2 --num-layers 2 --cpu-offload on && \
run ch05_405b_d4 --num-layers 4 --cpu-offload on && \
python tools/extrapolate_405b.py "$OUT" > "$OUT/extrapolation.json" && cat "$OUT/extrapolation.json"
