#!/usr/bin/env bash
# r4_s25: W^T kept with the in-backward optimizer -- GPU test (bitwise vs per-backward
# transposes, transpose count), then the 1-GPU bench --overlap-optimizer 0 vs 1, interleaved.
set -o pipefail
out=gpurun_out/r4_s25
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
    tests/test_kernels_gpu.py -k "weight_t or adamw" > "$out/pytest_wt.log" 2>&1 || { tail -40 "$out/pytest_wt.log"; exit 1; }
tail -1 "$out/pytest_wt.log"
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
    tests/test_engines_gpu.py tests/test_engines_rccl_gpu.py > "$out/pytest_eng.log" 2>&1 || { tail -40 "$out/pytest_eng.log"; exit 1; }
tail -1 "$out/pytest_eng.log"
ARGS="--steps 10 --warmup 3 --ref-steps 0 --fsdp-mem-steps 0"
for i in 1 2 3; do
  for v in 0 1; do
    timeout -k 10 300 python -u bench.py $ARGS --overlap-optimizer $v > "$out/bench_ov${v}_$i.log" 2>&1 \
        || { tail -20 "$out/bench_ov${v}_$i.log"; exit 1; }
    echo "overlap=$v run $i: $(grep -o '"ms_per_step": [0-9.]*' $out/bench_ov${v}_$i.log | head -1) $(grep -o '"final_loss": [0-9.]*' $out/bench_ov${v}_$i.log | head -1)"
  done
done
