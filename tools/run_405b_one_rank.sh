#!/bin/bash
# Chapter 05 with the reference's exact Llama-3.1-405B config (126 layers, b1 x 4096, FSDP
# transformer wrap, activation checkpointing, CPU offload) as ONE rank of its 64-GPU job
# (DTG_FAKE_WORLD=64: the other 63 ranks are a fake process group).  Measures that rank's
# memory and phase times without the communication.  Two offload layouts: parameters on the
# host too (the reference's CPUOffload(offload_params=True)) and parameter shard in HBM.
# Usage: gpurun --timeout 1200 -- bash tools/run_405b_one_rank.sh <tag>
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r405_one_rank}
mkdir -p $O
export TMPDIR=/tmp
( while true; do echo "[405b_one_rank] alive $(date +%T)"; sleep 30; done ) & HB=$!
trap 'kill $HB; rm -rf /tmp/dtg405r' EXIT
for op in on off; do
  rm -rf /tmp/dtg405r
  (cd 05-training-llama-405b && DTG_FAKE_WORLD=64 timeout -k 10 500 python -u train_llm.py -e r405 \
     -m meta-llama/Llama-3.1-405B -b 1 -s 4096 -d synthetic --num-workers 1 --save-dir /tmp/dtg405r \
     --ckpt-freq 100000 --max-steps 4 --log-freq 1 --cpu-offload on --offload-params $op \
     > $O/ch05_405b_w64_rank0_offload_params_$op.log 2>&1)
  rc=$?
  echo "offload-params=$op rc=$rc"
  grep -E "global_step': [34]," $O/ch05_405b_w64_rank0_offload_params_$op.log | grep -oE "'(time/forward|time/backward|time/update|time/total|peak_alloc_in_gb|peak_resv_in_gb|curr_alloc_in_gb)': [0-9.]+" | tr '\n' ' '; echo
  [ $rc -eq 0 ] || { tail -30 $O/ch05_405b_w64_rank0_offload_params_$op.log; exit $rc; }
done
