#!/usr/bin/env bash
# The 405B one-node recipes' GEMM shapes are not in the committed TunableOp table (hidden 16384):
# record them from short runs (depth 2, the per-layer shapes are depth-independent), then tune
# them offline one shape at a time (tools/tune_gemms.py; the results file is rewritten after
# every shape, so a time limit keeps the finished ones).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5_tune_405b}
mkdir -p "$O"
export TMPDIR=/tmp
rec() {  # name dir args...
  local name=$1 dir=$2; shift 2
  rm -rf /tmp/tune405
  (cd $dir && DTG_FAKE_WORLD=8 DTG_TUNABLEOP_RECORD=$O/untuned_$name.csv OMP_NUM_THREADS=16 timeout -k 10 240 \
     python -u train_llm.py -e tune -m meta-llama/Llama-3.1-405B --num-layers 2 -s 4096 -d synthetic --num-workers 1 \
     --save-dir /tmp/tune405 --ckpt-freq 100000 --max-steps 2 --log-freq 1 --cpu-offload on --offload-params off \
     --activation-checkpointing on "$@" > $O/rec_$name.log 2>&1) || { tail -20 $O/rec_$name.log; return 1; }
  echo "$name: $(cat $O/untuned_$name.csv* 2>/dev/null | grep -c Gemm) untuned GEMM calls recorded"
}
rec ch07_tp4 07-2d-parallel -b 4 --tp 4 && rec ch07_tp8 07-2d-parallel -b 8 --tp 8 && rec ch05 05-training-llama-405b -b 1 || exit 1
rm -rf /tmp/tune405
ls $O
timeout -k 10 1000 python -u tools/tune_gemms.py "$O/untuned_*" --out $O/tuned.csv --budget-s 780 --shape-timeout-s 150 \
    > $O/tune.log 2>&1; rc=$?
tail -30 $O/tune.log
exit $rc
