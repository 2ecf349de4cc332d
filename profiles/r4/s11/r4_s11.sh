#!/usr/bin/env bash
# r4_s11: token-major weight-gradient GEMM (csrc/kernels/dw_gemm.hip): numerics vs f32, then
# the microbench against hipBLASLt (TN pre-transposed, TN + transposes, NT) on the 8B dW shapes.
set -o pipefail
out=gpurun_out/r4_s11
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
    tests/test_dw_gemm_gpu.py > "$out/pytest_dwg.log" 2>&1 || { tail -40 "$out/pytest_dwg.log"; exit 1; }
tail -1 "$out/pytest_dwg.log"
timeout -k 10 300 python -u tools/bench_dw_gemm.py > "$out/bench_dwg.jsonl" 2> "$out/bench_dwg.err" \
    || { tail -20 "$out/bench_dwg.err"; exit 1; }
cat "$out/bench_dwg.jsonl"
# in-step A/B: hipBLASLt TN + transposes (0) vs the hand GEMM on token-major operands (1)
ARGS="--steps 10 --warmup 3 --ref-steps 0 --fsdp-mem-steps 0"
for i in 1 2; do
  for v in 0 1; do
    DTG_DW_GEMM=$v timeout -k 10 300 python -u bench.py $ARGS > "$out/bench_dwg${v}_$i.log" 2>&1 \
        || { tail -20 "$out/bench_dwg${v}_$i.log"; exit 1; }
    echo "dw_gemm=$v run $i: $(grep -o '"ms_per_step": [0-9.]*' $out/bench_dwg${v}_$i.log | head -1) $(grep -o '"final_loss": [0-9.]*' $out/bench_dwg${v}_$i.log | head -1)"
  done
done
export DTG_DW_GEMM=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/prof_dwg" -o run -- python -u bench.py --steps 3 --warmup 2 \
    --ref-steps 0 --fsdp-mem-steps 0 > "$out/prof_dwg.log" 2>&1 || { tail -20 "$out/prof_dwg.log"; exit 1; }
echo profiled
