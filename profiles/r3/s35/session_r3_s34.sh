#!/bin/bash
# Backward operand layouts at TP = 8 shapes (one rank of config 06, DTG_FAKE_WORLD=8):
# DTG_LINEAR_BWD=tn (transpose X and dY for every dW) vs auto (transpose only where the layer's
# output is at least as wide as its input), alternating on one box.
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/r3_s34
mkdir -p $O
export TMPDIR=/tmp
i=0
for m in tn auto tn auto; do
  i=$((i+1))
  DTG_LINEAR_BWD=$m DTG_FAKE_WORLD=8 timeout -k 10 240 python -u bench.py --gpus 8 --tp 8 --steps 10 --warmup 3 --fsdp-mem-steps 0 \
    > $O/tp8_${m}_$i.log 2>&1 || { tail -20 $O/tp8_${m}_$i.log; exit 1; }
  echo "tp8 $m: $(tail -1 $O/tp8_${m}_$i.log | grep -oE '"ms_per_step": [0-9.]+')"
done
