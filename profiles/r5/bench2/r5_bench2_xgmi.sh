#!/usr/bin/env bash
# bench.py's N > 1 diagnostics end to end on a small model (2 ranks sharing the GPU, gloo), so the
# xGMI child runs: its collective rows carry the cross-device checks (reduce-scatter max_rel_err
# vs the process group, all-gather equality) and the copy-engine ZeRO step its replica check.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5_bench2_xgmi}
mkdir -p "$O"
export TMPDIR=/tmp
( while true; do sleep 45; echo "[bench2x] alive"; done ) & HB=$!
trap 'kill $HB 2>/dev/null' EXIT
DTG_SHARED_DEVICE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29641 bench.py --gpus 2 --backend gloo --model llama-3.2-3b \
    --batch-size 2 --steps 2 --warmup 1 --fsdp-mem-steps 0 --coll-sweep-mb 16 --bucket-sweep-mb 256 \
    --sweep-steps 1 > "$O/bench2.log" 2>&1 || { tail -30 "$O/bench2.log"; exit 1; }
grep '^{' "$O/bench2.log" | tail -1 > "$O/bench2.json"
python3 -c "
import json; r=json.load(open('$O/bench2.json'))
print({k: r.get(k) for k in ('value','phase_s','wall_s','diagnostic_errors','replicas_consistent')})
x=r.get('xgmi_diag') or {}
print(json.dumps(x)[:1500])"
