#!/usr/bin/env bash
# r4_s01: new bench contract (fresh ids per step, loss band, reference-mode timers), ZeRO W^T
# rebuilt per bucket after the parameter all-gather (batched transpose on a side stream).
set -o pipefail
out=gpurun_out/r4_s01
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
    tests/test_kernels_gpu.py -k "transpose" tests/test_engines_rccl_gpu.py > "$out/pytest.log" 2>&1 \
    || { tail -40 "$out/pytest.log"; exit 1; }
tail -2 "$out/pytest.log"
timeout -k 10 300 python -u bench.py > "$out/bench_n1.log" 2>&1 || { tail -20 "$out/bench_n1.log"; exit 1; }
tail -1 "$out/bench_n1.log"
DTG_FAKE_WORLD=8 timeout -k 10 300 python -u bench.py --gpus 8 --fsdp-mem-steps 0 > "$out/bench_fake8.log" 2>&1 \
    || { tail -20 "$out/bench_fake8.log"; exit 1; }
tail -1 "$out/bench_fake8.log"
DTG_FAKE_WORLD=8 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/prof_fake8" -o run -- \
    python3 bench.py --gpus 8 --steps 3 --warmup 2 --fsdp-mem-steps 0 --ref-steps 0 > "$out/prof_fake8.log" 2>&1 \
    || { tail -20 "$out/prof_fake8.log"; exit 1; }
tail -1 "$out/prof_fake8.log"
echo done
