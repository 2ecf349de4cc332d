#!/bin/bash
# dK/dV kernel: staging items two ahead (PF=2) vs one ahead (PF=1), same box; numerics first.
mkdir -p gpurun_out/s51
( while true; do echo "[s51] alive $(date +%T)"; sleep 30; done ) & HB=$!
trap 'kill $HB' EXIT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "flash or attention" > gpurun_out/s51/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/s51/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
for pf in 1 2; do
  for shape in llama8b rime; do
    DTG_FA_KV_PF=$pf timeout -k 10 120 python tools/bench_attention.py --shape $shape --iters 30 > gpurun_out/s51/attn_${shape}_pf${pf}_r$rep.log 2>&1
    rc=$?; echo "pf=$pf $shape rc=$rc $(grep -o '"bwd_ms": [0-9.]*' gpurun_out/s51/attn_${shape}_pf${pf}_r$rep.log)"; [ $rc -eq 0 ] || exit $rc
  done
done
done
