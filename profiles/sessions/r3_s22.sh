#!/bin/bash
# One rank of a W-rank FSDP job (fake process group for the other ranks): chapter 04's memory
# table at W = 1, 2, 4 (control: real multi-rank runs exist) and 8 (the reference's row), with
# and without CPU offload, Llama-2-7B b10 and Llama-2-70B b2.
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/r3_s22
mkdir -p $O
export TMPDIR=/tmp
( while true; do echo "[s22] alive $(date +%T)"; sleep 30; done ) & HB=$!
trap 'kill $HB' EXIT
run() { timeout -k 10 300 python -u tools/fsdp_mem_one_rank.py "$@" >> $O/mem.jsonl 2>> $O/mem.err || { tail -20 $O/mem.err; exit 1; }; tail -1 $O/mem.jsonl | cut -c150-; }
for w in 1 2 4 8; do run --world $w; done
run --world 8 --cpu-offload
run --world 8 --model llama-2-70b --batch 2
run --world 8 --model llama-2-70b --batch 2 --cpu-offload
