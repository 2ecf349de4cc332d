#!/usr/bin/env bash
# r4_s45: kernel-time view of the fused RoPE backward: rocprofv3 kernel trace of the bench with
# DTG_FA_ROPE_FUSED=0 and =1 (dQ + dK/dV + RoPE kernel time per step).
set -o pipefail
out=gpurun_out/r4_s45
mkdir -p "$out"
export TMPDIR=/tmp
for v in 0 1; do
  DTG_FA_ROPE_FUSED=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/prof$v" -o run -- \
      python3 bench.py --steps 3 --warmup 2 --fsdp-mem-steps 0 --ref-steps 0 > "$out/prof$v.log" 2>&1 || { tail -20 "$out/prof$v.log"; exit 1; }
  tail -1 "$out/prof$v.log"
done
