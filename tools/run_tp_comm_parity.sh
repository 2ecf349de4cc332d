#!/bin/bash
# Chapter 06 (TP + SP) with 4 and 8 ranks sharing one MI355X (DTG_SHARED_DEVICE=1): the same
# run over each TP transport -- the process group's collectives (gloo here; RCCL on a node),
# the xGMI pull kernels, the xGMI copy engines -- must give the same losses.  Exact 8B width,
# --num-layers 2.  Then a rocprofv3 kernel trace of TP = 2 with a 5-chunk vocab-parallel loss
# head (tools/ce_overlap.py: is any stats gather waited on between chunks?).
# Usage: gpurun --timeout 1200 -- bash tools/run_tp_comm_parity.sh <tag>
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-tp_parity}
mkdir -p $O
export TMPDIR=/tmp
( while true; do echo "[tp_parity] alive $(date +%T)"; sleep 30; done ) & HB=$!
trap 'kill $HB; rm -rf /tmp/dtg_tpp' EXIT
for n in 4 8; do
  for comm in rccl xgmi xgmi-dma; do
    rm -rf /tmp/dtg_tpp
    (cd 06-tensor-parallel && DTG_SHARED_DEVICE=1 DTG_XGMI_TIMEOUT=60 timeout -k 10 300 python -u -m torch.distributed.run \
      --nnodes 1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2958$n train_llm.py -e tpp \
      -m meta-llama/Llama-3.1-8B --num-layers 2 -b 2 -s 1024 -d synthetic --num-workers 0 --log-freq 1 \
      --ckpt-freq 100000 --max-steps 4 --save-dir /tmp/dtg_tpp --tp-comm $comm --tp-comm-mb 64 \
      > $O/ch06_tp${n}_${comm}.log 2>&1)
    rc=$?
    echo "tp=$n comm=$comm rc=$rc losses: $(grep -oE "'running_loss': [0-9.]+" $O/ch06_tp${n}_${comm}.log | cut -d' ' -f2 | tr '\n' ' ')"
    [ $rc -eq 0 ] || { tail -30 $O/ch06_tp${n}_${comm}.log; exit $rc; }
  done
done
DTG_CE_CHUNK_GIB=0.125 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o %pid%_run -- \
  python3 tools/tp_overlap_gpu.py --chunks 2 --layers 2 --steps 2 --out $O/tp_overlap > $O/trace.log 2>&1 \
  || { tail -20 $O/trace.log; exit 1; }
python tools/ce_overlap.py $O/trace | tee $O/ce_overlap.txt
