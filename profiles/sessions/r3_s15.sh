#!/bin/bash
# Cold-operand (rotating 1 GiB buffer) TunableOp re-tune of every GEMM shape of the Llama-3-8B
# step (tools/llama8b_step_gemms.csv), then bench A/B: committed table vs the 3-shape cold table
# (r3_s14) vs the all-shape cold table.
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/r3_s15
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u tools/tune_gemms.py tools/llama8b_step_gemms.csv --out $O/cold_all.csv --retune --rotating-mb 1024 \
  --max-tuning-ms 30 --budget-s 600 --shape-timeout-s 200 > $O/tune.log 2>&1 || { tail -20 $O/tune.log; exit 1; }
grep "done" $O/tune.log
cp tunableop/tunableop_results_partial.csv $O/table_cold_all.csv
python tools/merge_tunableop.py $O/table_cold_all.csv $O/cold_all.csv || exit 1
cp tunableop/tunableop_results_partial.csv $O/table_cold3.csv
python tools/merge_tunableop.py $O/table_cold3.csv profiles/r3/s14/cold.csv || exit 1
for i in 1 2; do
  for v in base cold3 cold_all; do
    if [ $v = base ]; then unset DTG_TUNABLEOP_TABLE; else export DTG_TUNABLEOP_TABLE=$O/table_$v.csv; fi
    timeout -k 10 240 python -u bench.py --steps 10 --warmup 3 --fsdp-mem-steps 0 > $O/bench_${v}_$i.log 2>&1 \
      || { tail -20 $O/bench_${v}_$i.log; exit 1; }
    echo "table=$v run $i: $(tail -1 $O/bench_${v}_$i.log | grep -oE '"(ms_per_step|final_loss)": [0-9.]+' | tr '\n' ' ')"
  done
done
