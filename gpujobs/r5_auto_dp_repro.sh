#!/usr/bin/env bash
# Is chapter 02 over the copy engines (--dp-comm xgmi-dma, 2 ranks sharing the GPU) reproducible
# run to run, and does --dp-comm auto (calibration first) train like it?  Losses of 4 runs.
set -o pipefail
cd "$GRAFT_REPO_ROOT/02-distributed-data-parallel" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5_auto_dp}
mkdir -p "$O"
export TMPDIR=/tmp DTG_SHARED_DEVICE=1 DTG_XGMI_TIMEOUT=30 DTG_TRANSPORT_CALIBRATE=1
i=0
for v in xgmi-dma xgmi-dma auto auto rccl; do
  i=$((i+1))
  timeout -k 10 200 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port $((29700+i)) train_llm.py -e rep$i -m llama-tiny-d128 -b 2 -d synthetic --num-workers 0 \
      --log-freq 1 --ckpt-freq 1000 --max-steps 5 --save-dir /tmp/rep$i --dp-comm $v > "$O/run${i}_$v.log" 2>&1 \
      || { tail -20 "$O/run${i}_$v.log"; exit 1; }
  echo "$v: $(grep -oE "'running_loss': [0-9.eE+-]+" "$O/run${i}_$v.log" | cut -d' ' -f2 | paste -sd' ') $(grep -oE 'transport calibration.*' "$O/run${i}_$v.log" | head -1)"
  rm -rf /tmp/rep$i
done
