#!/bin/bash
# Full-step kernel profile of bench.py (Llama-3-8B, 1 GPU) after the attention rewrite.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s12
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/s12/trace -o run -- python3 bench.py --steps 3 --warmup 2 > gpurun_out/s12/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; tail -1 gpurun_out/s12/trace.log | cut -c1-300
exit $rc
