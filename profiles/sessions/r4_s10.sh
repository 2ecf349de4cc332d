#!/usr/bin/env bash
# r4_s10: weight-gradient GEMMs on a side stream (DTG_DW_STREAM=1): bitwise tests, then an
# interleaved same-box bench A/B (flagship 1-GPU step, off/on twice).  Kept only if >= 1% faster.
set -o pipefail
out=gpurun_out/r4_s13
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
    tests/test_dw_stream_gpu.py > "$out/pytest_dw.log" 2>&1 || { tail -40 "$out/pytest_dw.log"; exit 1; }
tail -1 "$out/pytest_dw.log"
ARGS="--steps 10 --warmup 3 --ref-steps 0 --fsdp-mem-steps 0"
for i in 1 2; do
  for v in 0 1; do
    DTG_DW_STREAM=$v timeout -k 10 300 python -u bench.py $ARGS > "$out/bench_dw${v}_$i.log" 2>&1 \
        || { tail -20 "$out/bench_dw${v}_$i.log"; exit 1; }
    echo "dw_stream=$v run $i: $(grep -o '"ms_per_step": [0-9.]*' $out/bench_dw${v}_$i.log | head -1)"
  done
done
