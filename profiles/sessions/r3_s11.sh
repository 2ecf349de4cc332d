#!/bin/bash
# Loss-head chunk size A/B (DTG_CE_CHUNK_GIB: 1 = 4 x 4096 rows, 2 = 2 x 8192, 4 = one 16384-row chunk).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r3_s11
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2; do
  for g in 1 2 4; do
    DTG_CE_CHUNK_GIB=$g timeout -k 10 240 python -u bench.py --steps 10 --warmup 3 --fsdp-mem-steps 0 \
      > $O/bench_ce${g}_$i.log 2>&1 || { tail -20 $O/bench_ce${g}_$i.log; exit 1; }
    echo "ce chunk ${g} GiB run $i: $(tail -1 $O/bench_ce${g}_$i.log | grep -oE '"(ms_per_step|peak_mem_gb|final_loss)": [0-9.]+' | tr '\n' ' ')"
  done
done
