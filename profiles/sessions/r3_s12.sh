#!/bin/bash
# adamw_t_ descriptor fix: GPU optimizer / engine tests, then the rime and GPT-2 chapters.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r3_s12
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engines_gpu.py -k "adamw or weight_t" -x -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/run_chapters_gpu.sh r3_s12 'ch00|ch01_gpt2$'
