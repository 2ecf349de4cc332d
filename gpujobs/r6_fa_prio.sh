#!/usr/bin/env bash
# Round 6 attention attempt: s_setprio around the forward's and dQ's MFMA phases (the wave issuing
# a GEMM block outranks its SIMD partner running softmax).  Builds: base (scratch: none), prio1,
# prio2 (DTG_EXTRA_HIPFLAGS=-DDTG_FA_PRIO=N).  Numerics of the variants first, then
# tools/bench_attention.py alternating the builds twice on three shapes.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r6_fa_prio}
mkdir -p "$O"
export TMPDIR=/tmp
for v in prio1 prio2; do
  DTG_NATIVE_SO=$GRAFT_REPO_ROOT/scratch/ab/${v}_C.so timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py \
      -k "flash_attn" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$O/pytest_$v.log" 2>&1 \
      || { tail -30 "$O/pytest_$v.log"; exit 1; }
  echo "$v numerics: $(tail -n 1 $O/pytest_$v.log)"
done
for i in 1 2; do
  for v in base prio1 prio2; do
    if [ "$v" = base ]; then env=""; else env="DTG_NATIVE_SO=$GRAFT_REPO_ROOT/scratch/ab/${v}_C.so"; fi
    for shape in llama8b rime long; do
      env $env timeout -k 10 120 python -u tools/bench_attention.py --shape $shape > "$O/${v}_${shape}_$i.log" 2>&1 \
          || { tail -20 "$O/${v}_${shape}_$i.log"; exit 1; }
      echo "$v $shape #$i $(tail -n 1 $O/${v}_${shape}_$i.log | grep -oE '"(fwd|bwd)_TFLOPs": [0-9.]+' | paste -sd' ')"
    done
  done
done
