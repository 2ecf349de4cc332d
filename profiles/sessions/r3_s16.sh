#!/bin/bash
# Bench A/B: committed TunableOp table vs the 3-shape and all-shape cold-operand re-tunes (r3_s14/15).
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/r3_s16
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2; do
  for v in base cold3 cold_all; do
    if [ $v = base ]; then unset DTG_TUNABLEOP_TABLE; else export DTG_TUNABLEOP_TABLE=$GRAFT_REPO_ROOT/tunableop/ab/$v.csv; fi
    timeout -k 10 240 python -u bench.py --steps 10 --warmup 3 --fsdp-mem-steps 0 > $O/bench_${v}_$i.log 2>&1 \
      || { tail -20 $O/bench_${v}_$i.log; exit 1; }
    echo "table=$v run $i: $(tail -1 $O/bench_${v}_$i.log | grep -oE '"(ms_per_step|final_loss)": [0-9.]+' | tr '\n' ' ')"
  done
done
