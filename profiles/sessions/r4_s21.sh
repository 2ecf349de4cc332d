#!/usr/bin/env bash
# r4_s21: chapters 02 (ZeRO) and 04 (FSDP) through the trainer CLI with --dp-comm xgmi-dma vs the
# process group, 2 ranks sharing the GPU.
set -o pipefail
out=gpurun_out/r4_s21
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_dp_comm_chapters_gpu.py > "$out/pytest_dpc.log" 2>&1 || { tail -40 "$out/pytest_dpc.log"; exit 1; }
tail -1 "$out/pytest_dpc.log"
