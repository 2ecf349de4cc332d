#!/bin/bash
# Ulysses and pipeline-parallel GPU tests (2 ranks sharing the GPU over gloo).
mkdir -p gpurun_out/s47
( while true; do echo "[s47] alive $(date +%T)"; sleep 30; done ) & HB=$!
trap 'kill $HB' EXIT
timeout -k 10 400 python -u -m pytest tests/test_pipeline_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/s47/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -6 gpurun_out/s47/pytest.log; exit $rc
