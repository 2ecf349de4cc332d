#!/usr/bin/env bash
# Same-box A/B of the tp 4 x dp 2 405B recipe (rank 0 of W = 8, depth 50) with the committed
# TunableOp table vs the table plus the tuned tp 4 shapes (gpurun_out/<tuned>.csv): A B A.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5_tp4_tune_ab}
TUNED=${2:-tunableop/untuned/tuned_405b_tp4.csv}
mkdir -p "$O"
export TMPDIR=/tmp
cp tunableop/tunableop_results_partial.csv $O/table_tuned.csv
python3 tools/merge_tunableop.py $O/table_tuned.csv $TUNED
( while true; do sleep 45; echo "[ab] alive"; done ) & HB=$!
trap 'kill $HB 2>/dev/null; rm -rf /tmp/tp4ab' EXIT
i=0
for v in base tuned base; do
  i=$((i+1))
  if [ $v = tuned ]; then export DTG_TUNABLEOP_TABLE=$O/table_tuned.csv; else unset DTG_TUNABLEOP_TABLE; fi
  rm -rf /tmp/tp4ab
  (cd 07-2d-parallel && DTG_FAKE_WORLD=8 OMP_NUM_THREADS=16 timeout -k 10 400 python -u train_llm.py -e ab \
     -m meta-llama/Llama-3.1-405B --num-layers 50 -b 4 -s 4096 -d synthetic --num-workers 1 --tp 4 \
     --save-dir /tmp/tp4ab --ckpt-freq 100000 --max-steps 4 --log-freq 1 --cpu-offload on --offload-params off \
     --activation-checkpointing on --pin-numa on --cpu-share 16 > $O/run${i}_$v.log 2>&1) || { tail -20 $O/run${i}_$v.log; exit 1; }
  echo "$v: $(grep -oE "'global_step': [234],|'time/total': [0-9.]+|'running_loss': [a-z0-9.]+" $O/run${i}_$v.log | paste -sd' ')"
done
