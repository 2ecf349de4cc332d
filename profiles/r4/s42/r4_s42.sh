#!/usr/bin/env bash
# r4_s42: rmsnorm_bwd grid size (DTG_RMSNORM_BWD_BLOCKS) -- bytes in flight per CU at 512 blocks
# are below what Little's law asks for at HBM latency; microbench incl. the dw column sums.
set -o pipefail
out=gpurun_out/r4_s42
mkdir -p "$out"
export TMPDIR=/tmp
for i in 1 2; do
  for b in 256 512 1024 2048; do
    DTG_RMSNORM_BWD_BLOCKS=$b timeout -k 10 180 python -u tools/bench_kernels.py --only rmsnorm_bwd --params 1e6 --layers 1 \
        > "$out/b${b}_$i.log" 2>&1 || { tail -20 "$out/b${b}_$i.log"; exit 1; }
    echo "blocks=$b $i $(grep rmsnorm_bwd $out/b${b}_$i.log | tail -1)"
  done
done
