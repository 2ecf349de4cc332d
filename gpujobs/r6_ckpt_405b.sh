#!/usr/bin/env bash
# Round 6: DCP checkpoint cost at exact Llama-3.1-405B width (chapter 05 recipe, W = 1, depth 1 --
# the embedding, the loss head and one decoder layer: 7.4 B parameters, a 44 GB checkpoint of
# bf16 parameters + both bf16 AdamW moments), CPU offload with the parameter shard in HBM.
# sync save vs --async-ckpt (snapshot into pinned host buffers, DCP written on a background
# thread over its own gloo group while step 3 trains), then the resume time.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r6_ckpt_405b}
mkdir -p $O
export TMPDIR=/tmp
S=/tmp/ck405
( while true; do echo "[ckpt405] alive $(date +%T) $(grep MemAvailable /proc/meminfo) $(du -sh $S 2>/dev/null | cut -f1)"; sleep 30; done ) & HB=$!
trap 'kill $HB; rm -rf $S' EXIT
df -h /tmp | tail -n 1
ARGS="-m meta-llama/Llama-3.1-405B --num-layers 1 -b 1 -s 4096 -d synthetic --num-workers 1 --save-dir $S \
  --log-freq 1 --cpu-offload on --offload-params off --activation-checkpointing on"
run() {  # <log tag> <experiment> <extra args>
  (cd 05-training-llama-405b && OMP_NUM_THREADS=16 timeout -k 10 500 python -u train_llm.py -e $2 $ARGS $3 \
     > $O/$1.log 2>&1)
  rc=$?
  echo "$1 rc=$rc: $(grep -oE 'training stalled [0-9.]+ s|finalize[^:]*: [0-9.]+ s|loaded in [0-9.]+ s|time/total.: [0-9.]+' $O/$1.log | paste -sd' ')"
  return $rc
}
run sync sync "--ckpt-freq 2 --max-steps 3" && du -sh $S/sync/checkpoint | tee $O/ckpt_size.txt && rm -rf $S/sync \
  && run async async "--ckpt-freq 2 --max-steps 3 --async-ckpt on" \
  && run resume async "--ckpt-freq 100 --max-steps 4 --async-ckpt on" || { tail -30 $O/*.log; exit 1; }
