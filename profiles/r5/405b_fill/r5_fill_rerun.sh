#!/usr/bin/env bash
# Rehearsals re-measured with the fake group's reduce-scatter / all-to-all outputs filled
# (utils/comm.py): 405B one node (ch05 FSDP, ch07 tp4 x dp2, ch07 tp8; depth 100) and the
# Llama-3-8B bench as rank 0 of dp8 / tp8.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r5_fill2}
O=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$O"
export TMPDIR=/tmp
for cfg in dp8 tp8; do
  extra=""; [ "$cfg" = "tp8" ] && extra="--tp 8"
  DTG_FAKE_WORLD=8 timeout -k 10 300 python3 bench.py --gpus 8 $extra --steps 10 --warmup 3 --ref-steps 0 ${EXTRA:-} \
      --fsdp-mem-steps 0 > "$O/bench_$cfg.log" 2>&1 || { tail -20 "$O/bench_$cfg.log"; exit 1; }
  tail -1 "$O/bench_$cfg.log" | cut -c1-400
done
bash tools/run_405b_node_w8.sh $tag 100 && bash gpujobs/r5_405b_2d.sh $tag "4:4:100 8:8:100"
