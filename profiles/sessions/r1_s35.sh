#!/bin/bash
# flash_attn.hip built with VGPR-form MFMA: numerics, attention micro-bench, step bench + profile.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s35
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_tp_xgmi_gpu.py -x -q --timeout 200 --timeout-method thread -k "flash or llama or tp2" > gpurun_out/s35/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/s35/pytest.log
[ $rc -eq 0 ] || exit $rc
for sh in llama8b rime; do
  timeout -k 10 200 python -u tools/bench_attention.py --shape $sh > gpurun_out/s35/attn_$sh.jsonl 2>&1
  rc=$?; echo "attn $sh rc=$rc"; grep '{' gpurun_out/s35/attn_$sh.jsonl | tail -2
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/s35/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/s35/bench.log | cut -c1-200
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/s35/prof -o run -- python3 bench.py --steps 3 --warmup 2 > gpurun_out/s35/prof.log 2>&1
rc=$?; echo "prof rc=$rc"
exit $rc
