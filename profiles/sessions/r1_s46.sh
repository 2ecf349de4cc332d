#!/bin/bash
# Ulysses and pipeline-parallel GPU tests (2 ranks sharing the GPU over gloo).
mkdir -p gpurun_out/s46
( while true; do echo "[s46] alive $(date +%T)"; sleep 30; done ) & HB=$!
trap 'kill $HB' EXIT
timeout -k 10 400 python -u -m pytest tests/test_ulysses_gpu.py tests/test_pipeline_gpu.py tests/test_cp_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/s46/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -6 gpurun_out/s46/pytest.log; exit $rc
