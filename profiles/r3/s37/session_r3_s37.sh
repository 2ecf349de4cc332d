#!/bin/bash
# Tune the GEMM shapes of TP = 4 and TP = 2 ranks (config 07's 2-D layouts; one rank via
# DTG_FAKE_WORLD=8) the committed table lacks, then A/B each with the committed vs merged table.
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/r3_s37
mkdir -p $O
export TMPDIR=/tmp
for tp in 4 2; do
  DTG_TUNABLEOP_RECORD=$O/untuned_tp$tp.csv DTG_FAKE_WORLD=8 timeout -k 10 240 python -u bench.py --gpus 8 --tp $tp --steps 2 --warmup 1 \
    --fsdp-mem-steps 0 > $O/record_tp$tp.log 2>&1 || { tail -20 $O/record_tp$tp.log; exit 1; }
done
ls $O
timeout -k 10 800 python -u tools/tune_gemms.py "$O/untuned_tp*.csv" --out $O/tuned.csv --rotating-mb 1024 \
  --max-tuning-ms 30 --budget-s 600 --shape-timeout-s 150 > $O/tune.log 2>&1 || { tail -20 $O/tune.log; exit 1; }
tail -2 $O/tune.log
cp tunableop/tunableop_results_partial.csv $O/table_new.csv
python tools/merge_tunableop.py $O/table_new.csv $O/tuned.csv || exit 1
for tp in 4 2; do
  for v in base new base new; do
    if [ $v = base ]; then unset DTG_TUNABLEOP_TABLE; else export DTG_TUNABLEOP_TABLE=$O/table_$v.csv; fi
    DTG_FAKE_WORLD=8 timeout -k 10 240 python -u bench.py --gpus 8 --tp $tp --steps 8 --warmup 3 --fsdp-mem-steps 0 \
      > $O/bench_tp${tp}_$v.log 2>&1 || { tail -20 $O/bench_tp${tp}_$v.log; exit 1; }
    echo "tp=$tp table=$v: $(tail -1 $O/bench_tp${tp}_$v.log | grep -oE '"ms_per_step": [0-9.]+')"
  done
done
unset DTG_TUNABLEOP_TABLE
timeout -k 10 400 python -u tools/check_tunableop.py --table $O/table_new.csv > $O/check.log 2>&1 || { tail -20 $O/check.log; exit 1; }
echo "check: $(grep -c '"ok": true' $O/check.log) ok, $(grep -c '"ok": false' $O/check.log || true) bad"
