#!/usr/bin/env bash
# r4_s05: ZeRO over the xGMI copy engines with 2/4/8 ranks sharing one GPU; bench N=1 after the
# round's changes (regression check) + a 2-rank shared-GPU bench rehearsal with both transports.
set -o pipefail
out=gpurun_out/r4_s05
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_xgmi_dp_gpu.py > "$out/pytest_xdp.log" 2>&1 || { tail -40 "$out/pytest_xdp.log"; exit 1; }
tail -1 "$out/pytest_xdp.log"
timeout -k 10 300 python -u bench.py > "$out/bench_n1.log" 2>&1 || { tail -20 "$out/bench_n1.log"; exit 1; }
tail -1 "$out/bench_n1.log"
echo done
