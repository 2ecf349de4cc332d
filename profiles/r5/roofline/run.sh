#!/usr/bin/env bash
# Round-5 step roofline at HEAD and the TP = 8 per-rank gap:
#  1. tools/step_pmc.sh: three rocprofv3 --pmc passes over bench.py N = 1 (1 warm-up + 1 timed
#     step, no reference-timer or FSDP-memory phase), summarised per step by tools/step_roofline.py
#  2. kernel trace (--kernel-trace --stats) of rank 0 of the 8-rank jobs, DTG_FAKE_WORLD=8:
#     dp8 ZeRO and tp8 (TP + SP), 2 warm-up + 3 timed steps each
#  3. the same two configs under torch.profiler (op x input shape table), separate runs
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r5_roofline}
O=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$O"
export TMPDIR=/tmp
bash tools/step_pmc.sh "$tag" || exit 1
for cfg in dp8 tp8; do
  extra=""; [ "$cfg" = "tp8" ] && extra="--tp 8"
  echo "[r5] kernel trace $cfg"
  DTG_FAKE_WORLD=8 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/trace_$cfg" -o run --output-format csv -- \
      python3 bench.py --gpus 8 $extra --steps 3 --warmup 2 --ref-steps 0 --fsdp-mem-steps 0 > "$O/trace_$cfg.log" 2>&1 \
      || { tail -20 "$O/trace_$cfg.log"; exit 1; }
  tail -1 "$O/trace_$cfg.log"
  echo "[r5] torch profile $cfg"
  DTG_FAKE_WORLD=8 timeout -k 10 300 python3 bench.py --gpus 8 $extra --steps 3 --warmup 2 --ref-steps 0 \
      --fsdp-mem-steps 0 --profile-steps 2 --profile-out "$O/torch_$cfg.txt" > "$O/torch_$cfg.log" 2>&1 \
      || { tail -20 "$O/torch_$cfg.log"; exit 1; }
  tail -1 "$O/torch_$cfg.log"
done

if [ "${FA64:-1}" = "1" ]; then
  echo "[r5] f64 forward numerics + A/B"
  timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "fwd_variants" -x -q --timeout 120 \
      --timeout-method thread > "$O/f64_pytest.log" 2>&1 || { tail -30 "$O/f64_pytest.log"; exit 1; }
  tail -2 "$O/f64_pytest.log"
  timeout -k 10 300 python -u tools/bench_attention.py --ab v0,f64 > "$O/f64_ab.jsonl" 2>&1 \
      || { tail -20 "$O/f64_ab.jsonl"; exit 1; }
  cat "$O/f64_ab.jsonl"
fi
echo "[r5] done"
