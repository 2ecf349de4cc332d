# Banded 1-D workgroup order (DTG_TILE_GROUP) for the transposing streaming kernels: numerics,
# kernel bandwidth per band width, then the full 8B step at the best candidates.
set -o pipefail
out=gpurun_out/s62
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "swiglu or transpose" -x -v --timeout 120 \
    --timeout-method thread -p no:cacheprovider > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for g in 0 4 8 16 32 0 8 16; do
  DTG_TILE_GROUP=$g timeout -k 10 200 python -u tools/bench_kernels.py > $out/kern_$g.log 2>&1 || { tail $out/kern_$g.log; exit 1; }
  echo "g=$g $(grep -E 'swiglu_bwd_t|transpose' $out/kern_$g.log | tr '\n' ' ')"
done
for g in 0 8 16 0 8 16; do
  DTG_TILE_GROUP=$g timeout -k 10 300 python -u bench.py > $out/bench_$g.log 2>&1 || { tail $out/bench_$g.log; exit 1; }
  echo "bench g=$g $(tail -1 $out/bench_$g.log | cut -c100-190)"
done
