#!/bin/bash
# bench.py as rank 0 of the driver's 8-GPU runs (DTG_FAKE_WORLD): dp8 ZeRO (the default N = 8
# command) and dp1 x tp8, each with the FSDP memory phase at W = 8 in-process.  Catches shape,
# shard-layout and memory problems of the N = 8 path before the driver runs it for real.
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/r3_s29
mkdir -p $O
export TMPDIR=/tmp
for n in 2 8; do
  DTG_FAKE_WORLD=$n timeout -k 10 420 python -u bench.py --gpus $n --steps 10 --warmup 3 > $O/bench_fake$n.log 2>&1 \
    || { tail -30 $O/bench_fake$n.log; exit 1; }
  echo "dp$n: $(tail -1 $O/bench_fake$n.log | cut -c1-900)"
done
DTG_FAKE_WORLD=8 timeout -k 10 420 python -u bench.py --gpus 8 --tp 8 --steps 10 --warmup 3 --fsdp-mem-steps 0 > $O/bench_fake8_tp8.log 2>&1 \
  || { tail -30 $O/bench_fake8_tp8.log; exit 1; }
echo "tp8: $(tail -1 $O/bench_fake8_tp8.log | cut -c1-700)"
