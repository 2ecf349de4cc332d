#!/usr/bin/env bash
# One GPU-box pass over the current tree: GPU test suite, driver smoke, default bench and a
# rocprofv3 kernel-time profile of the bench step.  Every GPU step has its own time limit and
# the chain stops at the first failure (no retries).
#
#   gpurun --timeout 1200 -- bash tools/gpu_check.sh s53
#   ONLY_PYTEST=1 ... (the suite alone) / PYTEST=0 ... (smoke, bench, profile)
set -o pipefail
tag=${1:-check}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
if [ "${PYTEST:-1}" = "1" ]; then
  echo "[gpu_check] pytest -m gpu"
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
      -p no:cacheprovider > "$out/pytest.log" 2>&1 || { tail -30 "$out/pytest.log"; exit 1; }
  tail -2 "$out/pytest.log"
  [ "${ONLY_PYTEST:-0}" = "1" ] && exit 0
fi
echo "[gpu_check] smoke"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 \
    || { tail -20 "$out/smoke.log"; exit 1; }
tail -1 "$out/smoke.log"
echo "[gpu_check] bench"
timeout -k 10 300 python -u bench.py > "$out/bench.log" 2>&1 || { tail -20 "$out/bench.log"; exit 1; }
tail -1 "$out/bench.log"
if [ "${PROFILE:-1}" = "1" ]; then
  echo "[gpu_check] rocprofv3 kernel stats"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/prof" -o run -- \
      python3 bench.py --steps 3 --warmup 2 > "$out/prof.log" 2>&1 || { tail -20 "$out/prof.log"; exit 1; }
  tail -1 "$out/prof.log"
fi
echo "[gpu_check] done"
