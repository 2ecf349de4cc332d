#!/usr/bin/env bash
# Hardware counters for every kernel of the headline training step (bench.py, Llama-3-8B,
# 16 x 1024, one MI355X): one rocprofv3 --pmc pass per counter group (TCC's FETCH_SIZE and
# WRITE_SIZE cannot share a pass), each its own run of the same 1 warm-up + 1 timed step.
# Summarise with tools/step_roofline.py.
#
#   gpurun --timeout 900 -- bash tools/step_pmc.sh r3_s30
set -o pipefail
tag=${1:-step_pmc}
out=gpurun_out/$tag/pmc
mkdir -p "$out"
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$out/avail.txt" 2>&1 || { tail -5 "$out/avail.txt"; exit 1; }
have() {
  local keep=()
  for c in "$@"; do grep -qw "$c" "$out/avail.txt" && keep+=("$c"); done
  echo "${keep[@]}"
}
PASS_A=$(have SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAVES \
              GRBM_GUI_ACTIVE GRBM_COUNT)
PASS_B=$(have FETCH_SIZE GRBM_GUI_ACTIVE)
PASS_C=$(have WRITE_SIZE GRBM_GUI_ACTIVE)
echo "[step_pmc] A: $PASS_A"; echo "[step_pmc] B: $PASS_B"; echo "[step_pmc] C: $PASS_C"
for p in A B C; do
  eval "ctrs=\$PASS_$p"
  [ -z "$ctrs" ] && continue
  echo "[step_pmc] pass $p"
  timeout -s KILL 300 rocprofv3 --pmc $ctrs -d "$out/$p" -o run --output-format csv -- \
      python3 bench.py --steps 1 --warmup 1 --fsdp-mem-steps 0 --ref-steps 0 > "$out/$p.log" 2>&1 \
      || { tail -20 "$out/$p.log"; exit 1; }
done
echo "[step_pmc] done"
