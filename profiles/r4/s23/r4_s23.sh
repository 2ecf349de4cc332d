#!/usr/bin/env bash
# r4_s23: chapter 05 (Llama-3.1-8B b1 x 4096, CPU offload) with and without the host gradient ring,
# parameters on the host and HBM-resident, interleaved, same box.
set -o pipefail
out=gpurun_out/r4_s23
mkdir -p "$out"
export TMPDIR=/tmp
cd 05-training-llama-405b || exit 1
TR="python -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29573"
for i in 1 2; do
  for ring in 0 4; do
    for op in on off; do
      timeout -k 10 300 $TR train_llm.py -e r$ring$op -m meta-llama/Llama-3.1-8B -b 1 -s 4096 -d synthetic \
          --save-dir /tmp/dtg_s23 --ckpt-freq 1000 --num-workers 2 --max-steps 6 --log-freq 2 \
          --offload-params $op --offload-grad-ring $ring > "../$out/ring${ring}_params${op}_$i.log" 2>&1 \
          || { tail -30 "../$out/ring${ring}_params${op}_$i.log"; exit 1; }
      echo "ring=$ring offload-params=$op run $i: $(grep global_step ../$out/ring${ring}_params${op}_$i.log | tail -1 | grep -oE "'(tok/s|time/backward|time/update)': [0-9.]+" | tr '\n' ' ')"
    done
  done
done
rm -rf /tmp/dtg_s23
