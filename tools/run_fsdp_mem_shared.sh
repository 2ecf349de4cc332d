#!/bin/bash
# Chapter 04's memory table (Llama-2-7B, b10 x 1024, size wrap 1e8, FULL_SHARD) at world W with
# every rank sharing the box's one MI355X (DTG_SHARED_DEVICE=1, gloo collectives).  Each rank's
# caching allocator is its own, so its valley / peak are what one of W GPUs would hold.  The
# timed phase runs a tiny model (the 8B DP step does not fit W times on one card).
# Usage: W=4 gpurun --timeout 1200 -- bash tools/run_fsdp_mem_shared.sh <tag>
cd "$GRAFT_REPO_ROOT" || exit 1
W=${W:-4}
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-fsdp_mem}
mkdir -p "$OUT"
export TMPDIR=/tmp
( while sleep 30; do echo "[fsdp_mem] alive $(date +%T)"; done ) &
HB=$!
trap "kill $HB" EXIT
DTG_SHARED_DEVICE=1 timeout -k 10 ${LIMIT:-900} python -u -m torch.distributed.run --nnodes 1 --nproc-per-node $W \
    --master-addr 127.0.0.1 --master-port 29575 bench.py --gpus $W --backend gloo \
    --model llama-tiny --batch-size 2 --seq-len 256 --steps 2 --warmup 1 --coll-sweep-mb "" \
    --fsdp-mem-steps ${FSDP_STEPS:-3} > "$OUT/fsdp_mem_w$W.log" 2>&1
rc=$?
echo "fsdp_mem W=$W rc=$rc"
tail -1 "$OUT/fsdp_mem_w$W.log" | grep -o '"fsdp_mem.*' || tail -30 "$OUT/fsdp_mem_w$W.log"
exit $rc
