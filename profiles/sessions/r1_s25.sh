#!/bin/bash
# FSDP engine bench + profile (1 GPU), rime chapter with the current kernels.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s25
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --parallel fsdp --steps 6 --warmup 2 > gpurun_out/s25/bench_fsdp.log 2>&1
rc=$?; echo "fsdp rc=$rc"; tail -1 gpurun_out/s25/bench_fsdp.log | cut -c1-250
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/s25/fsdp_prof -o run -- python3 bench.py --parallel fsdp --steps 3 --warmup 2 > gpurun_out/s25/fsdp_prof.log 2>&1
rc=$?; echo "fsdp prof rc=$rc"
[ $rc -eq 0 ] || exit $rc
cd 00-rime && timeout -k 10 400 python train_llm.py -e rime_gpu --max-steps 12 --log-freq 4 --ckpt-freq 1000 --save-dir ../gpurun_out/s25/outputs --num-workers 2 > ../gpurun_out/s25/rime.log 2>&1
rc=$?; cd ..; echo "rime rc=$rc"; grep -E "global_step|Error" gpurun_out/s25/rime.log | tail -2 | cut -c1-700
rm -rf gpurun_out/s25/outputs
exit $rc
