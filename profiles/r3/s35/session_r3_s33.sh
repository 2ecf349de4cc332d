#!/bin/bash
# Kernel-time profile of one TP = 8 rank of BASELINE config 06 (Llama-3-8B, 16 x 1024 per TP
# group; DTG_FAKE_WORLD=8, other ranks a fake process group): where a TP rank's compute goes.
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/r3_s33
mkdir -p $O
export TMPDIR=/tmp
DTG_FAKE_WORLD=8 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- \
  python3 bench.py --gpus 8 --tp 8 --steps 3 --warmup 2 --fsdp-mem-steps 0 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
tail -1 $O/prof.log | cut -c1-300
