#!/usr/bin/env bash
# TP = 8 vs dp8 rank kernel traces, re-taken on finite data (fake-world embedding fix,
# profiles/r5/fake_nan/): rank 0 of each 8-rank job, DTG_FAKE_WORLD=8, 2 warm-up + 3 timed steps.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5_tp8_gap2}
mkdir -p "$O"
export TMPDIR=/tmp
for cfg in dp8 tp8; do
  extra=""; [ "$cfg" = "tp8" ] && extra="--tp 8"
  DTG_FAKE_WORLD=8 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/trace_$cfg" -o run --output-format csv -- \
      python3 bench.py --gpus 8 $extra --steps 3 --warmup 2 --ref-steps 0 --fsdp-mem-steps 0 > "$O/trace_$cfg.log" 2>&1 \
      || { tail -20 "$O/trace_$cfg.log"; exit 1; }
  grep '^{' "$O/trace_$cfg.log" | tail -1 | cut -c1-300
done
