#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 4 --warmup 2 --parallel fsdp --tunableop off > gpurun_out/bench_fsdp1.log 2>&1
rc=$?; echo "bench(fsdp) rc=$rc"; tail -1 gpurun_out/bench_fsdp1.log | cut -c1-500
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
cd 00-rime && timeout -k 10 400 python train_llm.py -e rime_gpu --max-steps 12 --log-freq 4 --ckpt-freq 1000 --save-dir ../gpurun_out/outputs --num-workers 2 > ../gpurun_out/rime.log 2>&1
rc=$?; cd ..; echo "rime rc=$rc"; grep -E "global_step|Error" gpurun_out/rime.log | tail -3 | cut -c1-600
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 1000 python bench.py --steps 4 --warmup 2 --tunableop tune > gpurun_out/bench_tune.log 2> gpurun_out/bench_tune.err
rc=$?; echo "bench(tune) rc=$rc"; tail -1 gpurun_out/bench_tune.log | cut -c1-400; tail -3 gpurun_out/bench_tune.err
mkdir -p gpurun_out/tunableop && cp tunableop/*.csv gpurun_out/tunableop/ 2>/dev/null
exit $rc
