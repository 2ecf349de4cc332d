#!/usr/bin/env bash
# r4_s07: ZeRO + FSDP over the xGMI copy engines (2/4/8 ranks on one GPU), then the FSDP-phase A/B
# of HEAD vs the round-3 tree (build/r3head) on the same box (r4_s05 showed 1,788 ms vs 374).
set -o pipefail
out=gpurun_out/r4_s07
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -p no:cacheprovider \
    tests/test_xgmi_dp_gpu.py > "$out/pytest_xdp.log" 2>&1 || { tail -40 "$out/pytest_xdp.log"; exit 1; }
tail -1 "$out/pytest_xdp.log"
bash profiles/sessions/r4_s06.sh
mkdir -p "$out" && cp -r gpurun_out/r4_s06/* "$out/" 2>/dev/null
true
