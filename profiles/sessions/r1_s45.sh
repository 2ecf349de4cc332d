#!/bin/bash
# Full GPU suite (now with the context-parallel test) + smoke + default bench.
mkdir -p gpurun_out/s45
( while true; do echo "[s45] alive $(date +%T)"; sleep 30; done ) & HB=$!
trap 'kill $HB' EXIT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/s45/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/s45/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/s45/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/s45/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/s45/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/s45/bench.log; exit $rc
