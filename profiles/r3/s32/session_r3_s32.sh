#!/bin/bash
# SwiGLU-backward tile 64x128 (never actually run before: the knob's parser dropped it) vs the
# 64x64 default, in the full 8B step, alternating on one box; GPU tests for the tile knobs.
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/r3_s32
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "transpose2d or swiglu_bwd_t" -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
i=0
for t in 64x64 64x128 64x64 64x128 64x64 64x128; do
  i=$((i+1))
  DTG_SWIGLU_TILE=$t timeout -k 10 240 python -u bench.py --steps 10 --warmup 3 --fsdp-mem-steps 0 > $O/bench_${t}_$i.log 2>&1 \
    || { tail -20 $O/bench_${t}_$i.log; exit 1; }
  echo "tile=$t: $(tail -1 $O/bench_${t}_$i.log | grep -oE '"ms_per_step": [0-9.]+')"
done
