#!/bin/bash
# ch05 8B offload with loader workers: spawn context vs no pinning, to find the stall.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=$GRAFT_REPO_ROOT/gpurun_out/s44
mkdir -p $OUT
export TMPDIR=/tmp
( while sleep 20; do echo "[s44] alive"; done ) & HB=$!
cd 05-training-llama-405b
for v in "spawn:DTG_LOADER_CTX=spawn" "nopin:DTG_LOADER_PIN=0"; do
  tag=${v%%:*}; envs=${v#*:}
  env $envs timeout -k 10 150 python train_llm.py -e e8$tag -m meta-llama/Llama-3.1-8B -b 1 -s 4096 -d synthetic --save-dir $OUT/outputs --ckpt-freq 1000 --max-steps 2 --log-freq 1 --num-workers 2 > $OUT/$tag.log 2>&1
  echo "$tag rc=$? $(grep -oE "'global_step': [0-9]+|'time/forward': [0-9.]+|'time/backward': [0-9.]+|'time/update': [0-9.]+" $OUT/$tag.log | tail -4 | tr '\n' ' ')"
done
kill $HB; rm -rf $OUT/outputs
exit 0
