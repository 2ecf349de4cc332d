#!/usr/bin/env bash
# r4_s43: bench.py's N > 1 path on the GPU -- 2 ranks sharing one MI355X (gloo between them, as
# RCCL refuses two ranks per device), Llama-3.2-3B: the timed step, replica check, bucket sweep
# with the other ZeRO transport (xgmi-dma), xGMI collective rows; then the same with
# --dp-comm xgmi-dma as the timed transport.
set -o pipefail
out=gpurun_out/r4_s43
mkdir -p "$out"
export TMPDIR=/tmp
COMMON="--gpus 2 --backend gloo --model llama-3.2-3b --batch-size 4 --steps 3 --warmup 2 --fsdp-mem-steps 0 --coll-sweep-mb 16,64 --bucket-sweep-mb 64,256 --sweep-steps 2"
for dpc in rccl xgmi-dma; do
  DTG_SHARED_DEVICE=1 timeout -k 10 500 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 \
      --master-addr 127.0.0.1 --master-port 29611 bench.py $COMMON --dp-comm $dpc > "$out/bench2_$dpc.log" 2>&1 \
      || { tail -30 "$out/bench2_$dpc.log"; exit 1; }
  grep '^{' "$out/bench2_$dpc.log" | tail -1
done
