#!/usr/bin/env bash
# r4_s48: same-box check after r4_s47's slow bench (677 ms): fused RoPE off / on / off / on.
set -o pipefail
out=gpurun_out/r4_s48
mkdir -p "$out"
export TMPDIR=/tmp
for i in 1 2; do
  for v in 0 1; do
    DTG_FA_ROPE_FUSED=$v timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --fsdp-mem-steps 0 > "$out/bench_f${v}_$i.log" 2>&1 \
        || { tail -20 "$out/bench_f${v}_$i.log"; exit 1; }
    echo "bench fused=$v $i $(grep '^{' $out/bench_f${v}_$i.log | tail -1 | grep -o '"ms_per_step": [0-9.]*' | head -1)"
  done
done
