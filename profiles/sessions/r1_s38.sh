#!/bin/bash
# rime chapter regression hunt: VGPR-form flash build vs the previous codegen, same box.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=$GRAFT_REPO_ROOT/gpurun_out/s38
mkdir -p $OUT
export TMPDIR=/tmp
for v in novgpr vgpr; do
  if [ $v = novgpr ]; then export DTG_NATIVE_SO=$GRAFT_REPO_ROOT/lambda-labs_distributed-training-guide_amd/_C_novgpr.so; else unset DTG_NATIVE_SO; fi
  (cd 00-rime && timeout -k 10 300 python train_llm.py -e rime_$v -d synthetic --save-dir $OUT/outputs --ckpt-freq 1000 --num-workers 2 --max-steps 12 --log-freq 4 > $OUT/rime_$v.log 2>&1)
  rc=$?; echo "rime $v rc=$rc"; grep -oE "'global_step': 12|'tok/s': [0-9.]+|'time/forward': [0-9.]+|'time/backward': [0-9.]+" $OUT/rime_$v.log | tail -3 | tr '\n' ' '; echo
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 200 python -u tools/bench_attention.py --shape rime > $OUT/attn_rime_$v.jsonl 2>&1; grep '{' $OUT/attn_rime_$v.jsonl | tail -1
  timeout -k 10 200 python -u tools/bench_attention.py --shape long > $OUT/attn_long_$v.jsonl 2>&1; grep '{' $OUT/attn_long_$v.jsonl | tail -1
done
rm -rf $OUT/outputs
