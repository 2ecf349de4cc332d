#!/bin/bash
# Llama-3.1-405B on ONE 8-GPU MI355X node, measured as rank 0 of the W = 8 job (DTG_FAKE_WORLD=8:
# the other 7 ranks are a fake process group, so the rank's 1/8 shards, gathered units, offload
# traffic, host AdamW and compute are the real job's; the xGMI collectives are not).  Chapter 05's
# recipe at exact width: b1 x 4096, FSDP transformer wrap, activation checkpointing, CPU offload
# with the parameter shard resident in HBM (--offload-params off).  The rank is held to one
# rank's share of a node's cores (--cpu-share, OMP_NUM_THREADS) and to the GPU's NUMA node.
# Depths: the full 126 layers need ~406 GB of host state per rank (8 B per parameter: pinned bf16
# parameter + gradient shards, bf16 AdamW moments), beyond one box's 270 GiB command limit, so
# two reduced depths are measured and the per-layer costs extrapolated (tools/extrapolate_405b_w8.py).
# Usage: gpurun --timeout 1200 -- bash tools/run_405b_node_w8.sh <tag> [depths...]
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r405_w8}; shift
depths=${*:-8 56}
O=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p $O
export TMPDIR=/tmp
( while true; do echo "[405b_w8] alive $(date +%T) $(grep MemAvailable /proc/meminfo)"; sleep 30; done ) & HB=$!
trap 'kill $HB; rm -rf /tmp/dtg405w8' EXIT
grep -E "MemTotal|MemAvailable" /proc/meminfo > $O/meminfo_start.txt
nproc > $O/nproc.txt
SHARE=16
for d in $depths; do
  rm -rf /tmp/dtg405w8
  (cd 05-training-llama-405b && DTG_FAKE_WORLD=8 OMP_NUM_THREADS=$SHARE timeout -k 10 540 python -u train_llm.py \
     -e r405w8 -m meta-llama/Llama-3.1-405B --num-layers $d -b 1 -s 4096 -d synthetic --num-workers 1 \
     --save-dir /tmp/dtg405w8 --ckpt-freq 100000 --max-steps ${STEPS:-5} --log-freq 1 --cpu-offload on --offload-params off \
     --pin-numa on --cpu-share $SHARE --offload-grad-ring ${RING:-auto} ${EXTRA:-} > $O/ch05_405b_w8_rank0_depth$d.log 2>&1)
  rc=$?
  echo "depth=$d rc=$rc"
  grep -E "global_step': ($(seq -s'|' $(( ${STEPS:-5} - 1 )) ${STEPS:-5}))," $O/ch05_405b_w8_rank0_depth$d.log | grep -oE "'(time/forward|time/backward|time/update|time/total|peak_alloc_in_gb|peak_resv_in_gb|ac/layers|offload/[a-z0-9_]+|host/[a-z_]+)': [0-9.]+" | tr '\n' ' '; echo
  [ $rc -eq 0 ] || { tail -30 $O/ch05_405b_w8_rank0_depth$d.log; exit $rc; }
done
