#!/bin/bash
# HIP-graph captured training step: exactness vs eager, eager-vs-graph timing.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s28
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_graph_gpu.py tests/test_kernels_gpu.py -x -v --timeout 150 --timeout-method thread -k "graph or adamw" > gpurun_out/s28/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/s28/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u tools/bench_hipgraph.py > gpurun_out/s28/hipgraph.jsonl 2>&1
rc=$?; echo "bench rc=$rc"; cat gpurun_out/s28/hipgraph.jsonl | grep model
exit $rc
