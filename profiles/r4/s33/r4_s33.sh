#!/usr/bin/env bash
# r4_s33: DTG_FWD_XT (X^T taken in the forward, saved instead of X): bit-identity GPU tests, then
# an interleaved same-box bench A/B (same build, env switch).
set -o pipefail
out=gpurun_out/r4_s33
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
    tests/test_fwd_xt_gpu.py > "$out/pytest_fwd_xt.log" 2>&1 || { tail -40 "$out/pytest_fwd_xt.log"; exit 1; }
tail -1 "$out/pytest_fwd_xt.log"
for i in 1 2 3; do
  for v in 0 1; do
    DTG_FWD_XT=$v timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > "$out/bench_xt${v}_$i.log" 2>&1 \
        || { tail -20 "$out/bench_xt${v}_$i.log"; exit 1; }
    echo "bench xt=$v $i $(grep '^{' $out/bench_xt${v}_$i.log | tail -1 | grep -o '"ms_per_step": [0-9.]*\|"peak_gb": [0-9.]*\|"final_loss": [0-9.]*' | tr '\n' ' ')"
  done
done
