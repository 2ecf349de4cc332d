#!/usr/bin/env bash
# A/B: swiglu_bwd_t with one LDS buffer staged three times (DTG_SWIGLU_SEQ=1, 16.6 KB LDS, 6 waves
# per SIMD) against the three-buffer kernel (50 KB LDS, 3 workgroups per CU): numerics, kernel
# microbenchmark A B A B, then the 8B step A B A B, same box.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r6_swiglu_seq}
mkdir -p "$O"
export TMPDIR=/tmp
DTG_SWIGLU_SEQ=1 timeout -k 10 200 python -u -m pytest -x -q --timeout 100 --timeout-method thread -p no:cacheprovider \
    tests/test_kernels_gpu.py -k "swiglu" > "$O/pytest_seq.log" 2>&1 || { tail -30 "$O/pytest_seq.log"; exit 1; }
tail -1 "$O/pytest_seq.log"
for rep in 1 2; do
  for v in 0 1; do
    DTG_SWIGLU_SEQ=$v timeout -k 10 120 python -u tools/bench_kernels.py --only swiglu_bwd_t > "$O/kern_${v}_$rep.jsonl" 2>&1 \
        || { tail -20 "$O/kern_${v}_$rep.jsonl"; exit 1; }
    echo "seq=$v rep=$rep $(grep swiglu_bwd_t "$O/kern_${v}_$rep.jsonl")"
  done
done
for rep in 1 2; do
  for v in 0 1; do
    DTG_SWIGLU_SEQ=$v timeout -k 10 300 python -u bench.py > "$O/bench_${v}_$rep.log" 2>&1 || { tail -20 "$O/bench_${v}_$rep.log"; exit 1; }
    echo "seq=$v rep=$rep $(tail -1 "$O/bench_${v}_$rep.log" | grep -o '"ms_per_step": [0-9.]*\|"final_loss": [0-9.]*' | tr '\n' ' ')"
  done
done
