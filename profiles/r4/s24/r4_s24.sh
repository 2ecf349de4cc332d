#!/usr/bin/env bash
# r4_s24: 1-GPU bench with the AdamW update moved into the backward (--overlap-optimizer 1: each
# bucket's update on a side stream as soon as its gradients are final) vs the default, interleaved.
set -o pipefail
out=gpurun_out/r4_s24
mkdir -p "$out"
export TMPDIR=/tmp
ARGS="--steps 10 --warmup 3 --ref-steps 0 --fsdp-mem-steps 0"
for i in 1 2; do
  for v in 0 1; do
    timeout -k 10 300 python -u bench.py $ARGS --overlap-optimizer $v > "$out/bench_ov${v}_$i.log" 2>&1 \
        || { tail -20 "$out/bench_ov${v}_$i.log"; exit 1; }
    echo "overlap=$v run $i: $(grep -o '"ms_per_step": [0-9.]*' $out/bench_ov${v}_$i.log | head -1) $(grep -o '"final_loss": [0-9.]*' $out/bench_ov${v}_$i.log | head -1)"
  done
done
