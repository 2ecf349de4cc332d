#!/usr/bin/env bash
# r4_s06: the FSDP memory phase of bench.py ran 1,788 ms/step in r4_s05 vs 374 in r3: same-box A/B
# of the round-3 tree (build/r3head) against HEAD, FSDP phase only, twice each.
set -o pipefail
out=gpurun_out/r4_s06
mkdir -p "$out"
export TMPDIR=/tmp
ARGS="--steps 1 --warmup 1 --ref-steps 0 --fsdp-mem-steps 3 --fsdp-mem-world 0"
R3ARGS="--steps 1 --warmup 1 --fsdp-mem-steps 3 --fsdp-mem-world 0"
for i in 1 2; do
  timeout -k 10 240 python -u bench.py $ARGS > "$out/head_$i.log" 2>&1 || { tail -20 "$out/head_$i.log"; exit 1; }
  grep -o '"fsdp_mem": {[^}]*' "$out/head_$i.log" | grep -o '"ms_per_step": [0-9.]*' | sed "s/^/head $i /"
  (cd build/r3head && timeout -k 10 240 python -u bench.py $R3ARGS > "../../$out/r3_$i.log" 2>&1) || { tail -20 "$out/r3_$i.log"; exit 1; }
  grep -o '"fsdp_mem": {[^}]*' "$out/r3_$i.log" | grep -o '"ms_per_step": [0-9.]*' | sed "s/^/r3 $i /"
done
