#!/bin/bash
# Rewritten attention kernels: numerics, timings (dq occupancy 1 vs 2), kernel stats, bench.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s9
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -x > gpurun_out/s9/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/s9/pytest.log; [ $rc -ne 0 ] && exit $rc
for shape in llama8b rime gpt2; do
  for occ in 1 2; do
    DTG_FA_OCC=$occ timeout -k 10 120 python tools/bench_attention.py --shape $shape >> gpurun_out/s9/attn.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "attn $shape rc=$rc"; tail -3 gpurun_out/s9/attn.log; exit $rc; }
  done
done
grep shape gpurun_out/s9/attn.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/s9/trace -o run -- python3 tools/bench_attention.py --shape llama8b --iters 5 > gpurun_out/s9/trace.log 2>&1
echo "trace rc=$?"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA --kernel-trace -d gpurun_out/s9/pmc -o run -- python3 tools/bench_attention.py --shape llama8b --iters 2 > gpurun_out/s9/pmc.log 2>&1
echo "pmc rc=$?"
timeout -k 10 400 python bench.py --steps 6 --warmup 2 > gpurun_out/s9/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/s9/bench.log | cut -c1-300
exit $rc
