#!/bin/bash
# Same-box A/B of the transpose tile (64 vs 128) on the full 8B step, alternating runs.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s36
export TMPDIR=/tmp
for rep in 1 2; do
  for t in 64 128; do
    DTG_TRANSPOSE_TILE=$t timeout -k 10 300 python bench.py --steps 8 --warmup 3 > gpurun_out/s36/bench_t${t}_r$rep.log 2>&1
    rc=$?; echo "tile $t rep $rep rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/s36/bench_t${t}_r$rep.log)"
    [ $rc -eq 0 ] || exit $rc
  done
done
