#!/bin/bash
# Chapter 06 (TP = 8 + SP) as one rank of an 8-GPU node (DTG_FAKE_WORLD=8): step time without
# communication, then a rocprofv3 kernel table of the same run (where does TP's per-rank compute go?).
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/r3_s26
mkdir -p $O
export TMPDIR=/tmp
rm -rf /tmp/dtg_or
(cd 06-tensor-parallel && DTG_FAKE_WORLD=8 timeout -k 10 400 python -u train_llm.py -e tp8 -m meta-llama/Llama-3.1-8B -b 16 \
  -d synthetic --num-workers 1 --save-dir /tmp/dtg_or --ckpt-freq 100000 --max-steps 8 --log-freq 2 > $O/ch06_tp8.log 2>&1) \
  || { tail -30 $O/ch06_tp8.log; exit 1; }
grep mesh $O/ch06_tp8.log | cut -c1-150
echo "$(grep -E "global_step': 8," $O/ch06_tp8.log | grep -oE "'(tok/s|tok/s/gpu|peak_alloc_gb|time/forward|time/backward|time/update)': [0-9.]+" | tr '\n' ' ')"
rm -rf /tmp/dtg_or
cd 06-tensor-parallel && DTG_FAKE_WORLD=8 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- \
  python3 train_llm.py -e tp8p -m meta-llama/Llama-3.1-8B -b 16 -d synthetic --num-workers 1 --save-dir /tmp/dtg_or \
  --ckpt-freq 100000 --max-steps 4 --log-freq 2 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
echo profiled
