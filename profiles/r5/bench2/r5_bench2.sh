#!/usr/bin/env bash
# bench.py's N > 1 path at Llama-3-8B with every default diagnostic (transport calibration,
# collective sweep, bucket sweep, FSDP memory, xGMI child last), 2 ranks sharing one MI355X (gloo
# between them: RCCL refuses two ranks per device), batch 8 per rank so both fit in HBM.
# Records phase_s / wall_s against the 480 s deadline, and the xGMI child's cross-device checks.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5_bench2}
mkdir -p "$O"
export TMPDIR=/tmp
t0=$(date +%s)
# the gloo steps (host-staged 16 GB gradients) run ~14 s each with no output: keep the call alive
( while true; do sleep 50; echo "[bench2] alive $(( $(date +%s) - t0 )) s"; done ) & HB=$!
trap 'kill $HB 2>/dev/null' EXIT
DTG_SHARED_DEVICE=1 timeout -k 10 560 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29631 bench.py --gpus 2 --backend gloo --batch-size 8 \
    --steps 3 --warmup 1 > "$O/bench2.log" 2>&1 || { tail -30 "$O/bench2.log"; exit 1; }
echo "wall_outside_s=$(( $(date +%s) - t0 ))" | tee "$O/wall.txt"
grep '^{' "$O/bench2.log" | tail -1 > "$O/bench2.json"
python3 -c "
import json; r=json.load(open('$O/bench2.json'))
print({k: r.get(k) for k in ('value','ms_per_step','phase_s','wall_s','diagnostic_errors','replicas_consistent')})
x=r.get('xgmi_diag') or {}
print(json.dumps(x)[:1500])"
