#!/usr/bin/env bash
# Hardware counters of the hand dW GEMM variants next to hipBLASLt's TN / NT kernels on one
# Llama-3-8B dW shape (tools/bench_dw_gemm.py --only <shape>), one rocprofv3 --pmc pass per
# counter group; summarise with tools/pmc_summary.py <dir>/<pass>.
#
#   gpurun -- bash tools/dwg_pmc.sh r4_s13 gate_up
set -o pipefail
tag=${1:-dwg_pmc}
shape=${2:-gate_up}
out=gpurun_out/$tag/pmc_$shape
mkdir -p "$out"
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$out/avail.txt" 2>&1 || { tail -5 "$out/avail.txt"; exit 1; }
have() {
  local keep=()
  for c in "$@"; do grep -qw "$c" "$out/avail.txt" && keep+=("$c"); done
  echo "${keep[@]}"
}
PASS_A=$(have SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
              SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT)
PASS_B=$(have SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA \
              SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_SALU SQ_LDS_UNALIGNED_STALL)
PASS_C=$(have FETCH_SIZE GRBM_GUI_ACTIVE)
for p in A B C; do
  eval "ctrs=\$PASS_$p"
  [ -z "$ctrs" ] && continue
  echo "[dwg_pmc] $shape pass $p: $ctrs"
  timeout -s KILL 120 rocprofv3 --pmc $ctrs -d "$out/$p" -o run --output-format csv -- \
      python3 tools/bench_dw_gemm.py --only "$shape" --iters 3 > "$out/$p.log" 2>&1 \
      || { tail -20 "$out/$p.log"; exit 1; }
done
echo "[dwg_pmc] done"
