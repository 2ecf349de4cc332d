# FSDP after the gradient-accumulation fix and the overlapped host AdamW: chapter 05 (CPU
# offload) and chapter 04 on one MI355X, then the GPU suite.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=$GRAFT_REPO_ROOT/gpurun_out/s65
mkdir -p $OUT
export TMPDIR=/tmp
TR="python -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29565"
COMMON="-d synthetic --save-dir $OUT/outputs --ckpt-freq 1000 --num-workers 2"
run() {
  local name=$1 dir=$2; shift 2
  (cd $dir && timeout -k 10 400 "$@" > $OUT/$name.log 2>&1)
  local rc=$?
  echo "$name rc=$rc"; grep -E "global_step" $OUT/$name.log | tail -1 | grep -oE "'(global_step|running_loss|tok/s|peak_alloc_gb|peak_alloc_in_gb|time/forward|time/backward|time/update)': [0-9.e+-]+" | tr '\n' ' '; echo
  return $rc
}
( while sleep 30; do echo "[s65] alive $(date +%T)"; done ) &
HB=$!
trap "kill $HB" EXIT
run ch05_offload_8b 05-training-llama-405b $TR train_llm.py -e off8 -m meta-llama/Llama-3.1-8B -b 1 -s 4096 $COMMON --max-steps 4 --log-freq 2 || exit 1
run ch04_llama2_7b 04-fully-sharded-data-parallel $TR train_llm.py -e l27 -m meta-llama/Llama-2-7b-hf -b 10 $COMMON --max-steps 12 --log-freq 4 || exit 1
rm -rf $OUT/outputs
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
