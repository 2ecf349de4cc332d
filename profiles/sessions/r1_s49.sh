#!/bin/bash
# Attention kernels: where do the backward kernels' wave cycles go (parked vs issue-stalled vs active)?
mkdir -p gpurun_out/s49
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS --kernel-trace -d gpurun_out/s49/pmc -o run -- python3 tools/bench_attention.py --shape llama8b --iters 5 > gpurun_out/s49/pmc.log 2>&1
rc=$?; echo "pmc rc=$rc"; tail -3 gpurun_out/s49/pmc.log; exit $rc
