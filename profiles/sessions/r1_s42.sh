#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s42
export TMPDIR=/tmp
( while sleep 20; do echo "[s42] alive"; done ) & HB=$!
timeout -k 10 100 python -u tools/debug/fsdp_offload.py llama-3.2-3b > gpurun_out/s42/3b.log 2>&1; echo "3b rc=$?"; cat gpurun_out/s42/3b.log | grep "^\[" 
timeout -k 10 240 python -u tools/debug/fsdp_offload.py llama-3.1-8b > gpurun_out/s42/8b.log 2>&1; echo "8b rc=$?"; cat gpurun_out/s42/8b.log | grep "^\["
kill $HB
exit 0
