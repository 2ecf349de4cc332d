#!/usr/bin/env bash
# r4_s32: dK/dV loop without the 44 per-item AGPR->AGPR fragment copies (builtin vmcnt wait instead
# of the "+v" asm pin).  Attention GPU tests on HEAD, then interleaved A/Bs vs the previous build
# (build/ab/_C_base.so): attention microbench (8B + rime shapes) and the 8B bench step.
set -o pipefail
out=gpurun_out/r4_s32
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    tests/test_kernels_gpu.py -k "attn or flash or attention" > "$out/pytest_attn.log" 2>&1 || { tail -40 "$out/pytest_attn.log"; exit 1; }
tail -1 "$out/pytest_attn.log"
for i in 1 2 3; do
  for v in base head; do
    so=""; [ $v = base ] && so=build/ab/_C_base.so
    for sh in llama8b rime; do
      DTG_NATIVE_SO=$so timeout -k 10 120 python -u tools/bench_attention.py --shape $sh > "$out/attn_${v}_${sh}_$i.log" 2>&1 \
          || { tail -20 "$out/attn_${v}_${sh}_$i.log"; exit 1; }
      echo "attn $v $sh $i $(tail -1 $out/attn_${v}_${sh}_$i.log | cut -c1-200)"
    done
  done
done
for i in 1 2; do
  for v in base head; do
    so=""; [ $v = base ] && so=build/ab/_C_base.so
    DTG_NATIVE_SO=$so timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > "$out/bench_${v}_$i.log" 2>&1 \
        || { tail -20 "$out/bench_${v}_$i.log"; exit 1; }
    echo "bench $v $i $(grep '^{' $out/bench_${v}_$i.log | tail -1 | grep -o '"ms_per_step": [0-9.]*')"
  done
done
