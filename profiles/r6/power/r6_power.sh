#!/usr/bin/env bash
# Power and clock during the 8B bench step: samples amd-smi (power, clocks, usage) while
# bench.py runs 40 timed steps, to check the "GEMMs are power-limited" reading of the roofline
# (profiles/r6/roofline/: MFMA-busy 0.82 at an effective 1.78 GHz).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r6_power}
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 60 amd-smi static -g 0 --limit --json > "$O/static_limit.json" 2>&1 || true
timeout -k 10 60 amd-smi metric -g 0 --power --clock --usage --json > "$O/idle.json" 2>&1 || true
timeout -k 10 300 python -u bench.py --steps 40 --warmup 3 > "$O/bench.log" 2>&1 &
BP=$!
t0=$(date +%s.%N)
while kill -0 $BP 2>/dev/null; do
  t=$(date +%s.%N)
  echo "### t=$(python3 -c "print(round($t - $t0, 2))")" >> "$O/samples.txt"
  timeout -k 2 10 amd-smi metric -g 0 --power --clock --usage --json >> "$O/samples.txt" 2>&1
  sleep 0.2
done
wait $BP
rc=$?
tail -n 1 "$O/bench.log" | cut -c1-300
exit $rc
