#!/bin/bash
# Re-tune the three 8B GEMM shapes that run below 1.45 PF/s in the step with cold operands
# (TunableOp rotating buffer), then A/B the bench against the committed table.
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/r3_s14
mkdir -p $O
export TMPDIR=/tmp
printf "GemmTunableOp_BFloat16_TN,tn_4096_4096_16384_ld_16384_16384_4096\nGemmTunableOp_BFloat16_TN,tn_4096_6144_16384_ld_16384_16384_4096\nGemmTunableOp_BFloat16_TN,tn_4096_16384_4096_ld_4096_4096_4096\n" > $O/shapes.csv
timeout -k 10 600 python -u tools/tune_gemms.py $O/shapes.csv --out $O/cold.csv --retune --rotating-mb 1024 \
  --max-tuning-ms 30 --budget-s 480 --shape-timeout-s 200 > $O/tune.log 2>&1 || { tail -20 $O/tune.log; exit 1; }
grep "done" $O/tune.log
cp tunableop/tunableop_results_partial.csv $O/table_cold.csv
python tools/merge_tunableop.py $O/table_cold.csv $O/cold.csv || exit 1
for i in 1 2; do
  for v in base cold; do
    if [ $v = base ]; then unset DTG_TUNABLEOP_TABLE; else export DTG_TUNABLEOP_TABLE=$O/table_cold.csv; fi
    timeout -k 10 240 python -u bench.py --steps 10 --warmup 3 --fsdp-mem-steps 0 > $O/bench_${v}_$i.log 2>&1 \
      || { tail -20 $O/bench_${v}_$i.log; exit 1; }
    echo "table=$v run $i: $(tail -1 $O/bench_${v}_$i.log | grep -oE '"(ms_per_step|final_loss)": [0-9.]+' | tr '\n' ' ')"
  done
done
