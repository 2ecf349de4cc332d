#!/usr/bin/env bash
# Round 6 at HEAD: kernel-trace stats of the default bench (3 steps) and the per-step roofline
# (tools/step_pmc.sh: three rocprofv3 --pmc passes over one bench step), summarised on the box.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r6_profile}
O=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/trace" -o run --output-format csv -- \
    python3 bench.py --steps 3 --warmup 2 --fsdp-mem-steps 0 --ref-steps 0 > "$O/trace.log" 2>&1 \
    || { tail -20 "$O/trace.log"; exit 1; }
tail -n 1 "$O/trace.log"
bash tools/step_pmc.sh "$tag" || exit 1
python3 tools/step_roofline.py "$O/pmc" --window adamw_t --flops-gemm 7.38e14 --out "$O/step_roofline.md" \
    || exit 1
head -24 "$O/step_roofline.md"
find "$O/pmc" -name "*.csv" -size +20M -delete  # keep the merge small; the summary is the evidence
