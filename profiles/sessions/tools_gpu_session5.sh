#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for t in use off; do
  timeout -k 10 300 python bench.py --steps 6 --warmup 2 --tunableop $t > gpurun_out/bench_tun_$t.log 2>&1
  rc=$?; echo "bench(tunableop=$t) rc=$rc"; tail -1 gpurun_out/bench_tun_$t.log | cut -c1-300
  [ $rc -ne 0 ] && exit $rc
done
for par in zero ddp fsdp; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29600 \
    bench.py --gpus 2 --backend gloo --model llama-3.2-3b --batch-size 2 --seq-len 1024 --steps 3 --warmup 1 --parallel $par > gpurun_out/gloo2_$par.log 2>&1
  rc=$?; echo "gloo x2 ($par) rc=$rc"; grep -E "metric|Error" gpurun_out/gloo2_$par.log | tail -2 | cut -c1-300
  [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof2 -o run -- python3 bench.py --steps 3 --warmup 2 > gpurun_out/prof2.log 2>&1
rc=$?; echo "rocprof rc=$rc"
exit $rc
