#!/usr/bin/env bash
# r4_s03: host gradient ring (GPU test) + 405B W = 8 rank 0 with the ring at depths 8 and 80.
set -o pipefail
out=gpurun_out/r4_s03
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
    tests/test_engines_rccl_gpu.py -k "offload" > "$out/pytest.log" 2>&1 || { tail -30 "$out/pytest.log"; exit 1; }
tail -1 "$out/pytest.log"
RING=auto bash tools/run_405b_node_w8.sh r4_s03 8 80
