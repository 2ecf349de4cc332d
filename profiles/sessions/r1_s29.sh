#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s29
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/debug/graph_gpt2_order.py > gpurun_out/s29/dbg.log 2>&1; echo rc=$?; grep -v amdgpu gpurun_out/s29/dbg.log | cut -c1-250 | tail -20; exit 0
rc=$?; echo "rc=$rc"; grep -v amdgpu.ids gpurun_out/s29/g_only.jsonl | tail -4
timeout -k 10 300 python -u tools/bench_hipgraph.py --models gpt2 --batches 1 --modes eager,hipgraph > gpurun_out/s29/e_g.jsonl 2>&1
rc=$?; echo "rc=$rc"; grep -v amdgpu.ids gpurun_out/s29/e_g.jsonl | tail -4
timeout -k 10 300 python -u tools/bench_hipgraph.py --models gpt2 --batches 1 --modes eager,hipgraph --steps 3 > gpurun_out/s29/e_g3.jsonl 2>&1
rc=$?; echo "rc=$rc"; grep -v amdgpu.ids gpurun_out/s29/e_g3.jsonl | tail -4
exit $rc
