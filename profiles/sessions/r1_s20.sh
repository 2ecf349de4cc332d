#!/bin/bash
# Optimizer-in-backward on the GPU: bench with and without, 2-rank gloo engine rehearsal on one GPU.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s20
export TMPDIR=/tmp
for ov in 1 0; do
  timeout -k 10 400 python bench.py --steps 10 --warmup 3 --overlap-optimizer $ov > gpurun_out/s20/bench_ov$ov.log 2>&1
  rc=$?; echo "bench ov=$ov rc=$rc"; tail -1 gpurun_out/s20/bench_ov$ov.log | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
done
DTG_SHARED_DEVICE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 2 --backend gloo --model llama-tiny-d128 --batch-size 4 --seq-len 512 > gpurun_out/s20/bench_gloo2.log 2>&1
rc=$?; echo "gloo2 rc=$rc"; grep metric gpurun_out/s20/bench_gloo2.log | cut -c1-300
exit $rc
