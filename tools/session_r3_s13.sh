#!/bin/bash
# In-step A/B of hipBLASLt solutions for the three GEMM shapes that run below 1.45 PF/s in the
# 8B step (o_proj dW, qkv dW, o_proj fwd/dX): sustained sweep -> candidate tables -> bench each.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r3_s13
mkdir -p $O
export TMPDIR=/tmp
( while true; do echo "[s13] alive $(date +%T)"; sleep 30; done ) & HB=$!
trap 'kill $HB' EXIT
[ -x build/gemm_sustained ] || { echo "build/gemm_sustained missing"; exit 1; }
for spec in tn_4096_4096_16384_ld_16384_16384_4096 tn_4096_6144_16384_ld_16384_16384_4096 tn_4096_16384_4096_ld_4096_4096_4096; do
  timeout -k 10 240 build/gemm_sustained $spec 0.3 6 >> $O/sustained.jsonl 2>> $O/sustained.err
  rc=$?; echo "$spec rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python tools/tunableop_variants.py $O/sustained.jsonl --k 3 --out $O/tables > $O/variants.txt || exit 1
cat $O/variants.txt
for i in 1 2; do
  for v in base v0 v1 v2; do
    if [ $v = base ]; then unset DTG_TUNABLEOP_TABLE; else export DTG_TUNABLEOP_TABLE=$O/tables/$v.csv; fi
    timeout -k 10 240 python -u bench.py --steps 10 --warmup 3 --fsdp-mem-steps 0 > $O/bench_${v}_$i.log 2>&1 \
      || { tail -20 $O/bench_${v}_$i.log; exit 1; }
    echo "table=$v run $i: $(tail -1 $O/bench_${v}_$i.log | grep -oE '"(ms_per_step|final_loss)": [0-9.]+' | tr '\n' ' ')"
  done
done
