#!/usr/bin/env bash
# Round 6: the 2-D + offload recipe at EXACT Llama-3.1-405B width with REAL collectives --
# 4 ranks share the GPU (DTG_SHARED_DEVICE=1, gloo) as tp 2 x dp 2, depth 2, b1 x 4096 per rank,
# AC, CPU offload with the parameter shard resident -- against the single-process oracle at the
# same width and depth (b2 x 4096), both loading the same safetensors weights
# (tools/rehearse_405b_shared.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r6_405b_shared}
L=${2:-2}
mkdir -p $O
export TMPDIR=/tmp
W=/tmp/w405_d$L
( while true; do echo "[405b_shared] alive $(date +%T) $(grep MemAvailable /proc/meminfo) $(du -sh $W 2>/dev/null | cut -f1)"; sleep 30; done ) & HB=$!
trap 'kill $HB; rm -rf $W' EXIT
df -h /tmp | tee $O/df.txt
T="python -u tools/rehearse_405b_shared.py"
timeout -k 10 300 $T prep --dir $W --layers $L > $O/prep.log 2>&1 || { tail -20 $O/prep.log; exit 1; }
tail -1 $O/prep.log
OMP_NUM_THREADS=16 timeout -k 10 400 $T run --dir $W --layers $L --tp 1 --batch 2 --out $O/oracle.json \
    > $O/oracle.log 2>&1 || { tail -20 $O/oracle.log; exit 1; }
tail -1 $O/oracle.log
DTG_SHARED_DEVICE=1 OMP_NUM_THREADS=4 timeout -k 10 700 python -u -m torch.distributed.run --nnodes 1 \
    --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29533 tools/rehearse_405b_shared.py run --dir $W \
    --layers $L --tp 2 --batch 1 --out $O/twod.json > $O/twod.log 2>&1 || { tail -30 $O/twod.log; exit 1; }
tail -1 $O/twod.log
$T compare $O/oracle.json $O/twod.json | tee $O/compare.json
