#!/usr/bin/env bash
# Round-5 GPU suite with per-test durations, then smoke and the default bench.
set -o pipefail
out=gpurun_out/${1:-r5_suite}
mkdir -p "$out"
export TMPDIR=/tmp
t0=$(date +%s)
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --durations=40 --timeout 300 --timeout-method thread \
    -p no:cacheprovider > "$out/pytest.log" 2>&1 || { tail -40 "$out/pytest.log"; exit 1; }
echo "suite_s=$(( $(date +%s) - t0 ))" | tee "$out/suite_time.txt"
tail -45 "$out/pytest.log"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 || { tail -20 "$out/smoke.log"; exit 1; }
tail -1 "$out/smoke.log"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > "$out/bench.log" 2>&1 || { tail -20 "$out/bench.log"; exit 1; }
tail -1 "$out/bench.log"
