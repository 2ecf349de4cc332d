#!/usr/bin/env bash
# r4_s28: kernel trace of rank 0 of a 4-rank ZeRO run over the xGMI copy engines (shared GPU).
set -o pipefail
out=gpurun_out/r4_s28
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 700 python -u tools/trace_xgmi_dp_ranks.py --world 4 --out "$out/trace" > "$out/launcher.log" 2>&1 \
    || { tail -20 "$out/launcher.log"; tail -30 "$out/trace/rank0.log"; exit 1; }
tail -2 "$out/launcher.log"; grep '^{' "$out/trace/rank0.log" | tail -1 | cut -c1-400
