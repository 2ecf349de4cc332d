#!/bin/bash
# ch05 trainer 8B offload: which setting stalls the first step (loader workers / TunableOp)?
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=$GRAFT_REPO_ROOT/gpurun_out/s43
mkdir -p $OUT
export TMPDIR=/tmp
( while sleep 20; do echo "[s43] alive"; done ) & HB=$!
cd 05-training-llama-405b
for v in "w0:--num-workers 0" "tunoff:--tunableop off --num-workers 2"; do
  tag=${v%%:*}; extra=${v#*:}
  timeout -k 10 120 python train_llm.py -e e8$tag -m meta-llama/Llama-3.1-8B -b 1 -s 4096 -d synthetic --save-dir $OUT/outputs --ckpt-freq 1000 --max-steps 2 --log-freq 1 $extra > $OUT/$tag.log 2>&1
  echo "$tag rc=$? $(grep -oE "'global_step': [0-9]+|'time/forward': [0-9.]+|'time/backward': [0-9.]+|'time/update': [0-9.]+" $OUT/$tag.log | tail -4 | tr '\n' ' ')"
done
kill $HB; rm -rf $OUT/outputs
exit 0
