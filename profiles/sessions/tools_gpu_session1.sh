#!/bin/bash
# GPU session: fragment probes, kernel numerics tests, flagship bench, rocprofv3 kernel stats.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
hipcc --offload-arch=gfx950 -O2 -o /tmp/probe tests/native/probe_fragments.hip 2>/dev/null
timeout -k 10 120 /tmp/probe > gpurun_out/probe.log 2>&1; echo "probe rc=$?"; cat gpurun_out/probe.log
timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: pytest crashed"; exit $rc; fi
timeout -k 10 600 python bench.py --steps 5 --warmup 2 > gpurun_out/bench1.log 2>&1
rc=$?
echo "bench rc=$rc"; tail -2 gpurun_out/bench1.log
exit $rc
