#!/usr/bin/env bash
# Same-box step A/B of the register-blocked streaming kernels (transpose2d, adamw_t_) against the
# LDS-tiled ones: bench.py N = 1, alternating B A B A, then the engine / optimizer GPU tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5_step_ab}
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -k "adamw or weight_t or transpose" -x -q --timeout 120 \
    --timeout-method thread -p no:cacheprovider > "$O/pytest.log" 2>&1 || { tail -30 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
for i in 1 2; do
  for v in lds reg; do
    if [ "$v" = lds ]; then env="DTG_TRANSPOSE_TILE=64 DTG_ADAMT_KERNEL=lds DTG_ADAMT_TC=128"; else env=""; fi
    env $env timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --fsdp-mem-steps 0 --ref-steps 0 \
        > "$O/bench_${v}_$i.log" 2>&1 || { tail -20 "$O/bench_${v}_$i.log"; exit 1; }
    echo "$v #$i $(grep -oE '"ms_per_step": [0-9.]+|"final_loss": [0-9.]+' "$O/bench_${v}_$i.log" | paste -sd' ')"
  done
done
