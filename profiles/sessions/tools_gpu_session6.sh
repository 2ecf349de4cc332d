#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/rocprof_counters.txt 2>&1 || true
for shape in llama8b rime gpt2; do
  for v in 1 2; do
    DTG_FA_BWD=$v timeout -k 10 120 python tools/bench_attention.py --shape $shape >> gpurun_out/attn_bench.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "attn bench $shape v$v rc=$rc"; tail -3 gpurun_out/attn_bench.log; exit $rc; }
  done
done
cat gpurun_out/attn_bench.log | grep shape
for par in zero ddp fsdp; do
  DTG_SHARED_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29600 \
    bench.py --gpus 2 --backend gloo --model llama-3.2-3b --batch-size 2 --seq-len 1024 --steps 3 --warmup 1 --parallel $par --tunableop off > gpurun_out/gloo2_$par.log 2>&1
  rc=$?; echo "gloo x2 ($par) rc=$rc"; grep -E "metric|Error" gpurun_out/gloo2_$par.log | tail -2 | cut -c1-300
  [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
done
exit 0
