#!/bin/bash
# rime chapter: commit 67968de (rime 45.8k tok/s in s25) vs HEAD, same box, alternating.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=$GRAFT_REPO_ROOT/gpurun_out/s40
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  for tree in _ab_old .; do
    tag=$( [ $tree = . ] && echo head || echo old )
    (cd $tree/00-rime && timeout -k 10 300 python train_llm.py -e r_${tag}_$rep -d synthetic --save-dir $OUT/outputs --ckpt-freq 1000 --num-workers 2 --max-steps 12 --log-freq 4 > $OUT/rime_${tag}_$rep.log 2>&1)
    rc=$?; echo "$tag rep $rep rc=$rc $(grep -oE "'tok/s': [0-9.]+|'time/forward': [0-9.]+|'time/backward': [0-9.]+" $OUT/rime_${tag}_$rep.log | tail -3 | tr '\n' ' ')"
    [ $rc -eq 0 ] || exit $rc
  done
done
rm -rf $OUT/outputs
