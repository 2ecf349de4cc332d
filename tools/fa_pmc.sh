#!/usr/bin/env bash
# Hardware-counter passes over the flash-attention kernels (fwd, bwd_dq, bwd_dkdv) at the 8B
# bench shape and the rime packed shape.  One rocprofv3 --pmc run per counter group (the SQ
# block holds 8 counters per pass, TCC 4, GRBM 2); counters the device does not list are
# dropped before a pass starts.  Summarise with tools/pmc_summary.py.
#
#   gpurun --timeout 900 -- bash tools/fa_pmc.sh r2_s17
set -o pipefail
tag=${1:-fa_pmc}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$out/avail.txt" 2>&1 || { tail -5 "$out/avail.txt"; exit 1; }

have() {  # keep only counters present in the device's list
  local keep=()
  for c in "$@"; do grep -qw "$c" "$out/avail.txt" && keep+=("$c"); done
  echo "${keep[@]}"
}

PASS_A=$(have SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
              SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT)
PASS_B=$(have SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA \
              SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_SALU SQ_LDS_UNALIGNED_STALL)
PASS_C=$(have FETCH_SIZE GRBM_GUI_ACTIVE)
echo "[fa_pmc] A: $PASS_A"
echo "[fa_pmc] B: $PASS_B"
echo "[fa_pmc] C: $PASS_C"

for shape in llama8b rime; do
  mkdir -p "$out/$shape"
  for p in A B C; do
    eval "ctrs=\$PASS_$p"
    [ -z "$ctrs" ] && continue
    echo "[fa_pmc] $shape pass $p"
    timeout -s KILL 120 rocprofv3 --pmc $ctrs -d "$out/$shape/$p" -o run --output-format csv -- \
        python3 tools/bench_attention.py --shape "$shape" --iters 2 > "$out/$shape/$p.log" 2>&1 \
        || { tail -20 "$out/$shape/$p.log"; exit 1; }
  done
done
echo "[fa_pmc] timing (unprofiled)"
for shape in llama8b rime; do
  timeout -k 10 120 python3 tools/bench_attention.py --shape "$shape" --iters 20 >> "$out/timing.jsonl" 2>"$out/timing.err" \
      || { tail -20 "$out/timing.err"; exit 1; }
done
cat "$out/timing.jsonl"
echo "[fa_pmc] done"
