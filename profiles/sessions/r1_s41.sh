#!/bin/bash
# Chapter 05 (FSDP + CPU offload + AC) on the GPU: tiny model timing, then an 8B run with a
# faulthandler stack dump (SIGUSR1) after 90 s to see where the step spends its time.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=$GRAFT_REPO_ROOT/gpurun_out/s41
mkdir -p $OUT
export TMPDIR=/tmp
COMMON="-d synthetic --save-dir $OUT/outputs --ckpt-freq 1000 --num-workers 2"
cd 05-training-llama-405b
timeout -k 10 200 python train_llm.py -e t -m llama-tiny-d128 -b 2 -s 512 $COMMON --max-steps 6 --log-freq 2 > $OUT/tiny.log 2>&1
echo "tiny rc=$? $(grep -oE "'global_step': [0-9]+|'time/forward': [0-9.]+|'time/backward': [0-9.]+|'time/update': [0-9.]+" $OUT/tiny.log | tail -4 | tr '\n' ' ')"
python train_llm.py -e e8 -m meta-llama/Llama-3.1-8B -b 1 -s 4096 $COMMON --max-steps 3 --log-freq 1 > $OUT/8b.log 2>&1 &
PID=$!
for i in 1 2 3; do sleep 30; echo "waiting $i"; done
kill -USR1 $PID; sleep 5
kill -USR1 $PID; sleep 5
kill $PID; sleep 3; kill -9 $PID 2>/dev/null
grep -oE "'global_step': [0-9]+|'time/forward': [0-9.]+|'time/backward': [0-9.]+|'time/update': [0-9.]+" $OUT/8b.log | tail -4 | tr '\n' ' '
rm -rf $OUT/outputs
exit 0
