#!/bin/bash
# rime chapter kernel profile: GPU busy time vs the synchronised phase timers.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=$GRAFT_REPO_ROOT/gpurun_out/s39
mkdir -p $OUT
export TMPDIR=/tmp
cd 00-rime && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 train_llm.py -e rime_prof -d synthetic --save-dir $OUT/outputs --ckpt-freq 1000 --num-workers 2 --max-steps 12 --log-freq 4 > $OUT/rime.log 2>&1
rc=$?; cd ..; echo "rc=$rc"; grep -oE "'global_step': 12|'tok/s': [0-9.]+|'time/forward': [0-9.]+|'time/backward': [0-9.]+|'time/data': [0-9.]+" $OUT/rime.log | tail -4 | tr '\n' ' '
rm -rf $OUT/outputs
exit $rc
