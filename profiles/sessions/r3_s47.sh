#!/bin/bash
# One rank of the N = 8 ZeRO bench (DTG_FAKE_WORLD=8): --overlap-optimizer 0 vs 1 (per-bucket
# AdamW + parameter all-gather on a side stream during backward), alternating; compute only.
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/r3_s47
mkdir -p $O
export TMPDIR=/tmp
i=0
for v in 0 1 0 1; do
  i=$((i+1))
  DTG_FAKE_WORLD=8 timeout -k 10 240 python -u bench.py --gpus 8 --steps 10 --warmup 3 --fsdp-mem-steps 0 --overlap-optimizer $v \
    > $O/dp8_ov${v}_$i.log 2>&1 || { tail -20 $O/dp8_ov${v}_$i.log; exit 1; }
  echo "overlap=$v: $(tail -1 $O/dp8_ov${v}_$i.log | grep -oE '"(ms_per_step|peak_mem_gb)": [0-9.]+' | tr '\n' ' ')"
done
