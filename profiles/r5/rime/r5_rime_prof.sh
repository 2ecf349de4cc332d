#!/usr/bin/env bash
# Chapter 00 (rime: Llama-3.2-3B-rime, packed 8192-token rows) kernel breakdown: 12 steps under
# rocprofv3 --kernel-trace --stats, then the same run unprofiled for tok/s.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5_rime_prof}
mkdir -p "$O"
export TMPDIR=/tmp
cd 00-rime || exit 1
timeout -k 10 300 python -u train_llm.py -e rime -d synthetic:packed --save-dir /tmp/rime_out --ckpt-freq 1000 \
    --num-workers 2 --max-steps 16 --log-freq 4 > "$O/rime.log" 2>&1 || { tail -20 "$O/rime.log"; exit 1; }
grep -oE "'tok/s': [0-9.]+" "$O/rime.log" | tail -2
rm -rf /tmp/rime_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/trace" -o run --output-format csv -- \
    python3 -u train_llm.py -e rime -d synthetic:packed --save-dir /tmp/rime_out --ckpt-freq 1000 \
    --num-workers 2 --max-steps 12 --log-freq 4 > "$O/rime_prof.log" 2>&1 || { tail -20 "$O/rime_prof.log"; exit 1; }
rm -rf /tmp/rime_out
head -25 "$O/trace/run_kernel_stats.csv" | cut -c1-160
