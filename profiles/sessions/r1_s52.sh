#!/bin/bash
# After the dK/dV wait fix: PMC pass on attention + the 8B bench.
mkdir -p gpurun_out/s52
export TMPDIR=/tmp
( while true; do echo "[s52] alive $(date +%T)"; sleep 30; done ) & HB=$!
trap 'kill $HB' EXIT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS --kernel-trace -d gpurun_out/s52/pmc -o run -- python3 tools/bench_attention.py --shape llama8b --iters 5 > gpurun_out/s52/pmc.log 2>&1
rc=$?; echo "pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/s52/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/s52/bench.log | cut -c1-400; exit $rc
