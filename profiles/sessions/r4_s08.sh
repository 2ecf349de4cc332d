#!/usr/bin/env bash
# r4_s08: (1) FSDP over the xGMI copy engines, 2/4/8 ranks on one GPU (ZeRO: r4_s05); (2) FSDP-phase A/B,
# HEAD vs the round-3 tree, same box; (3) attention A/B: dK/dV mask only on the halves that need
# it (HEAD _C.so) vs the masked-every-half build (build/ab/_C_base.so), interleaved processes.
set -o pipefail
out=gpurun_out/r4_s08
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
    tests/test_dw_gemm_gpu.py > "$out/pytest_dwg.log" 2>&1 || { tail -40 "$out/pytest_dwg.log"; exit 1; }
tail -1 "$out/pytest_dwg.log"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_xgmi_dp_gpu.py -k fsdp > "$out/pytest_xdp.log" 2>&1 || { tail -40 "$out/pytest_xdp.log"; exit 1; }
tail -1 "$out/pytest_xdp.log"
ARGS="--steps 1 --warmup 1 --ref-steps 0 --fsdp-mem-steps 3 --fsdp-mem-world 0"
R3ARGS="--steps 1 --warmup 1 --fsdp-mem-steps 3 --fsdp-mem-world 0"
for i in 1 2; do
  timeout -k 10 240 python -u bench.py $ARGS > "$out/fsdp_head_$i.log" 2>&1 || { tail -20 "$out/fsdp_head_$i.log"; exit 1; }
  grep -o '"fsdp_mem": {[^}]*' "$out/fsdp_head_$i.log" | grep -o '"ms_per_step": [0-9.]*' | sed "s/^/fsdp head $i /"
  (cd build/r3head && timeout -k 10 240 python -u bench.py $R3ARGS > "../../$out/fsdp_r3_$i.log" 2>&1) || { tail -20 "$out/fsdp_r3_$i.log"; exit 1; }
  grep -o '"fsdp_mem": {[^}]*' "$out/fsdp_r3_$i.log" | grep -o '"ms_per_step": [0-9.]*' | sed "s/^/fsdp r3 $i /"
done
for i in 1 2; do
  for v in base head; do
    so=""; [ $v = base ] && so=build/ab/_C_base.so
    for sh in llama8b rime; do
      DTG_NATIVE_SO=$so timeout -k 10 120 python -u tools/bench_attention.py --shape $sh > "$out/attn_${v}_${sh}_$i.log" 2>&1 \
          || { tail -20 "$out/attn_${v}_${sh}_$i.log"; exit 1; }
      echo "attn $v $sh $i $(tail -1 $out/attn_${v}_${sh}_$i.log)"
    done
  done
done
