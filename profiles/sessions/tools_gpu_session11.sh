#!/bin/bash
# Attention: numerics + timings after the tile-loop unroll and threshold masks; end-to-end bench.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s11
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -x > gpurun_out/s11/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/s11/pytest.log; [ $rc -ne 0 ] && exit $rc
for shape in llama8b rime gpt2 long; do
  timeout -k 10 120 python tools/bench_attention.py --shape $shape >> gpurun_out/s11/attn.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "attn $shape rc=$rc"; tail -3 gpurun_out/s11/attn.log; exit $rc; }
done
grep shape gpurun_out/s11/attn.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/s11/trace -o run -- python3 tools/bench_attention.py --shape llama8b --iters 5 > gpurun_out/s11/trace.log 2>&1
echo "trace rc=$?"
timeout -k 10 400 python bench.py --steps 8 --warmup 2 > gpurun_out/s11/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/s11/bench.log | cut -c1-300
exit $rc
