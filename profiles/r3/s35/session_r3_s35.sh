#!/bin/bash
# Tune the GEMM shapes of a TP = 8 rank (BASELINE config 06, one rank via DTG_FAKE_WORLD=8) that
# the committed table lacks (cold operands, rotating 1 GiB), then A/B the TP = 8 rank step with
# the committed vs the merged table, alternating.
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/r3_s35
mkdir -p $O
export TMPDIR=/tmp
DTG_TUNABLEOP_RECORD=$O/untuned.csv DTG_FAKE_WORLD=8 timeout -k 10 240 python -u bench.py --gpus 8 --tp 8 --steps 2 --warmup 1 \
  --fsdp-mem-steps 0 > $O/record.log 2>&1 || { tail -20 $O/record.log; exit 1; }
ls $O; cat $O/untuned*.csv | sort -u | wc -l
timeout -k 10 800 python -u tools/tune_gemms.py "$O/untuned*.csv" --out $O/tuned.csv --rotating-mb 1024 \
  --max-tuning-ms 30 --budget-s 660 --shape-timeout-s 150 > $O/tune.log 2>&1 || { tail -20 $O/tune.log; exit 1; }
tail -3 $O/tune.log
cp tunableop/tunableop_results_partial.csv $O/table_tp8.csv
python tools/merge_tunableop.py $O/table_tp8.csv $O/tuned.csv || exit 1
for i in 1 2; do
  for v in base tp8; do
    if [ $v = base ]; then unset DTG_TUNABLEOP_TABLE; else export DTG_TUNABLEOP_TABLE=$O/table_$v.csv; fi
    DTG_FAKE_WORLD=8 timeout -k 10 240 python -u bench.py --gpus 8 --tp 8 --steps 10 --warmup 3 --fsdp-mem-steps 0 \
      > $O/bench_${v}_$i.log 2>&1 || { tail -20 $O/bench_${v}_$i.log; exit 1; }
    echo "table=$v run $i: $(tail -1 $O/bench_${v}_$i.log | grep -oE '"ms_per_step": [0-9.]+')"
  done
done
