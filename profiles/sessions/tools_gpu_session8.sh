#!/bin/bash
# Per-kernel times and PMC counters of the attention kernels (llama8b shape).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s8
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/s8/trace -o run -- python3 tools/bench_attention.py --shape llama8b --iters 5 > gpurun_out/s8/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/s8/trace.log; exit $rc; }
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS --kernel-trace -d gpurun_out/s8/pmc1 -o run -- python3 tools/bench_attention.py --shape llama8b --iters 2 > gpurun_out/s8/pmc1.log 2>&1
rc=$?; echo "pmc1 rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/s8/pmc1.log; exit $rc; }
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA --kernel-trace -d gpurun_out/s8/pmc2 -o run -- python3 tools/bench_attention.py --shape llama8b --iters 2 > gpurun_out/s8/pmc2.log 2>&1
rc=$?; echo "pmc2 rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/s8/pmc2.log; exit $rc; }
find gpurun_out/s8 -name "*.csv" | head -20
exit 0
