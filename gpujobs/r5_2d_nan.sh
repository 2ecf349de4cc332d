#!/usr/bin/env bash
# Where does the 405B-width 2-D rehearsal (DTG_FAKE_WORLD=8) turn NaN at step 4?  A few layers at
# exact width, 8 steps, --check-finite grad; with and without CPU offload.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5_2d_nan}
mkdir -p "$O"
export TMPDIR=/tmp
for cfg in ${CFGS:-on off}; do
  rm -rf /tmp/dtg2dnan
  (cd 07-2d-parallel && DTG_FAKE_WORLD=8 OMP_NUM_THREADS=16 timeout -k 10 300 python -u train_llm.py \
     -e nan2d -m meta-llama/Llama-3.1-405B --num-layers ${DEPTH:-4} -b 4 -s 4096 -d synthetic --num-workers 1 \
     --tp 4 --save-dir /tmp/dtg2dnan --ckpt-freq 100000 --max-steps ${STEPS:-8} --log-freq 1 --cpu-offload $cfg \
     --offload-params off --activation-checkpointing on --check-finite grad > $O/tp4_offload_$cfg.log 2>&1) || { tail -30 $O/tp4_offload_$cfg.log; exit 1; }
  echo "offload=$cfg"; grep -oE "'running_loss': [a-z0-9.]+|check-finite.*" $O/tp4_offload_$cfg.log | cut -c1-300
done
rm -rf /tmp/dtg2dnan
