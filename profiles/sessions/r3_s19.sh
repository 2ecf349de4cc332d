#!/bin/bash
# Attention kernel before / after the dQ tile-body refactor (248 VGPRs: two waves per SIMD):
# same box, alternating, kernel timing and the bench step.  build/_C_fa_old.so = HEAD with the
# round-3-start flash_attn.hip.
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/r3_s19
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2 3; do
  for v in old new; do
    if [ $v = old ]; then export DTG_NATIVE_SO=$GRAFT_REPO_ROOT/build/_C_fa_old.so; else unset DTG_NATIVE_SO; fi
    for shape in llama8b rime long; do
      timeout -k 10 120 python -u tools/bench_attention.py --shape $shape --iters 20 >> $O/attn_$v.jsonl 2>>$O/attn.err \
        || { tail -20 $O/attn.err; exit 1; }
    done
  done
done
grep -h shape $O/attn_old.jsonl | sed 's/^/old /'; grep -h shape $O/attn_new.jsonl | sed 's/^/new /'
for i in 1 2; do
  for v in old new; do
    if [ $v = old ]; then export DTG_NATIVE_SO=$GRAFT_REPO_ROOT/build/_C_fa_old.so; else unset DTG_NATIVE_SO; fi
    timeout -k 10 240 python -u bench.py --steps 10 --warmup 3 --fsdp-mem-steps 0 > $O/bench_${v}_$i.log 2>&1 \
      || { tail -20 $O/bench_${v}_$i.log; exit 1; }
    echo "fa=$v run $i: $(tail -1 $O/bench_${v}_$i.log | grep -oE '"ms_per_step": [0-9.]+')"
  done
done
