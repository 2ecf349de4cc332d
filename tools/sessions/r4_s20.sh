#!/usr/bin/env bash
# r4_s20: dW GEMM variants 8 and 9 (register-staged, hipBLASLt structure) next to 5: numerics,
# microbench, and -- if the microbench puts the best within 8 % of the transpose + TN path -- the
# interleaved same-box step A/B with DTG_DW_GEMM=1 and the faster of variants 4 / 5.
set -o pipefail
out=gpurun_out/r4_s20
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
    tests/test_dw_gemm_gpu.py > "$out/pytest_dwg.log" 2>&1 || { tail -40 "$out/pytest_dwg.log"; exit 1; }
tail -1 "$out/pytest_dwg.log"
timeout -k 10 300 python -u tools/bench_dw_gemm.py > "$out/bench_dwg.jsonl" 2> "$out/bench_dwg.err" \
    || { tail -20 "$out/bench_dwg.err"; exit 1; }
tail -1 "$out/bench_dwg.jsonl"
best=$(python -c "import json;d=json.loads(open('$out/bench_dwg.jsonl').read().splitlines()[-1])['per_layer_ms'];v=min(('5','8','9'),key=lambda k:d['hand_v'+k]);print(v, int(d['hand_v'+v]<1.08*d['tn_total']))")
echo "best variant / go: $best"
var=${best% *}; go=${best#* }
if [ "$go" = "1" ]; then
  ARGS="--steps 10 --warmup 3 --ref-steps 0 --fsdp-mem-steps 0"
  for i in 1 2; do
    for v in 0 1; do
      DTG_DW_GEMM=$v DTG_DWG_VARIANT=$var timeout -k 10 300 python -u bench.py $ARGS > "$out/bench_dwg${v}_$i.log" 2>&1 \
          || { tail -20 "$out/bench_dwg${v}_$i.log"; exit 1; }
      echo "dw_gemm=$v run $i: $(grep -o '"ms_per_step": [0-9.]*' $out/bench_dwg${v}_$i.log | head -1)"
    done
  done
fi
timeout -k 10 200 bash tools/dwg_pmc.sh r4_s20 gate_up > "$out/pmc.log" 2>&1 || { tail -5 "$out/pmc.log"; exit 1; }
echo done
