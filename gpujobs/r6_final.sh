#!/usr/bin/env bash
# Round 6 at HEAD: the whole GPU suite with per-test durations, smoke, and the default bench
# twice (what the driver runs at round end).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r6_final}
mkdir -p "$O"
export TMPDIR=/tmp
t0=$(date +%s)
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --durations=40 --timeout 300 --timeout-method thread \
    -p no:cacheprovider > "$O/pytest.log" 2>&1 || { tail -40 "$O/pytest.log"; exit 1; }
echo "suite_s=$(( $(date +%s) - t0 ))" | tee "$O/suite_time.txt"
tail -n 2 "$O/pytest.log"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { tail -20 "$O/smoke.log"; exit 1; }
tail -n 1 "$O/smoke.log"
for i in 1 2; do
  timeout -k 10 300 python -u bench.py > "$O/bench_$i.log" 2>&1 || { tail -20 "$O/bench_$i.log"; exit 1; }
  tail -n 1 "$O/bench_$i.log"
done
