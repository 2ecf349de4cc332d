#!/bin/bash
# Split-query dK/dV for KV-head-poor grids: tests, kernel A/B (TP = 8 / 4 shapes and the 8B
# shape), chapter 06 TP = 8 as one rank before / after.
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/r3_s27
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "flash or attention" -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python -u tools/bench_attention.py --ab-bwd DTG_FA_KV_SPLIT=1,2,4 --ab-tolerant > $O/ab_bwd.log 2>&1 || { tail -20 $O/ab_bwd.log; exit 1; }
grep case $O/ab_bwd.log
for v in 1 0; do
  rm -rf /tmp/dtg_or
  (cd 06-tensor-parallel && DTG_FA_KV_SPLIT=$v DTG_FAKE_WORLD=8 timeout -k 10 300 python -u train_llm.py -e tp8 -m meta-llama/Llama-3.1-8B \
    -b 16 -d synthetic --num-workers 1 --save-dir /tmp/dtg_or --ckpt-freq 100000 --max-steps 8 --log-freq 2 > $O/ch06_tp8_split$v.log 2>&1) \
    || { tail -30 $O/ch06_tp8_split$v.log; exit 1; }
  echo "split=$v (0 = auto): $(grep -E "global_step': 8," $O/ch06_tp8_split$v.log | grep -oE "'(tok/s/gpu|time/forward|time/backward)': [0-9.]+" | tr '\n' ' ')"
done
timeout -k 10 240 python -u bench.py --steps 10 --warmup 3 --fsdp-mem-steps 0 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
echo "bench: $(tail -1 $O/bench.log | grep -oE '"ms_per_step": [0-9.]+')"
