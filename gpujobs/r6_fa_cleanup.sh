#!/usr/bin/env bash
# Round 6: after removing the killed attention variants (f64 / p64 / narrow / wide / qlds /
# concurrent backward) and reading the backward's launch knobs once: the whole GPU suite with
# durations, then a same-box step A/B against the round-5 build (scratch/ab/r5_C.so via
# DTG_NATIVE_SO), alternating new / r5 twice; the step's final loss must be bitwise equal.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r6_fa_cleanup}
mkdir -p "$O"
export TMPDIR=/tmp
t0=$(date +%s)
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --durations=40 --timeout 300 --timeout-method thread \
    -p no:cacheprovider > "$O/pytest.log" 2>&1 || { tail -40 "$O/pytest.log"; exit 1; }
echo "suite_s=$(( $(date +%s) - t0 ))" | tee "$O/suite_time.txt"
tail -3 "$O/pytest.log"
for i in 1 2; do
  for v in new r5; do
    if [ "$v" = r5 ]; then env="DTG_NATIVE_SO=$GRAFT_REPO_ROOT/scratch/ab/r5_C.so"; else env=""; fi
    env $env timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --fsdp-mem-steps 0 --ref-steps 0 \
        > "$O/bench_${v}_$i.log" 2>&1 || { tail -20 "$O/bench_${v}_$i.log"; exit 1; }
    echo "$v #$i $(grep -oE '"ms_per_step": [0-9.]+|"final_loss": [0-9.]+' "$O/bench_${v}_$i.log" | paste -sd' ')"
  done
done
timeout -k 10 200 python -u tools/bench_attention.py --shape llama8b > "$O/attn_llama8b.log" 2>&1 && tail -2 "$O/attn_llama8b.log"
