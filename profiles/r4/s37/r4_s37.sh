#!/usr/bin/env bash
# r4_s37: dK/dV with V in LDS at two waves per SIMD (DTG_FA_KV_VLDS=1; 58 VGPRs spilled by hipcc
# at the 256-register budget): attention GPU tests under the variant, then interleaved microbench.
set -o pipefail
out=gpurun_out/r4_s37
mkdir -p "$out"
export TMPDIR=/tmp
DTG_FA_KV_VLDS=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    tests/test_kernels_gpu.py -k "attn or flash or attention" > "$out/pytest_attn_vlds.log" 2>&1 || { tail -40 "$out/pytest_attn_vlds.log"; exit 1; }
tail -1 "$out/pytest_attn_vlds.log"
for i in 1 2; do
  for v in 0 1; do
    for sh in llama8b rime llama8b-tp8; do
      DTG_FA_KV_VLDS=$v timeout -k 10 120 python -u tools/bench_attention.py --shape $sh > "$out/attn_v${v}_${sh}_$i.log" 2>&1 \
          || { tail -20 "$out/attn_v${v}_${sh}_$i.log"; exit 1; }
      echo "attn vlds=$v $sh $i $(tail -1 $out/attn_v${v}_${sh}_$i.log | grep -o '"bwd_ms": [0-9.]*')"
    done
  done
done
