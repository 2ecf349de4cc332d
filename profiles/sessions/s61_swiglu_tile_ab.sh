set -o pipefail
mkdir -p gpurun_out/s61
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k swiglu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/s61/pytest.log 2>&1 || { tail -30 gpurun_out/s61/pytest.log; exit 1; }
tail -1 gpurun_out/s61/pytest.log
for tt in 64 128 64 128; do
  DTG_SWIGLU_TT=$tt timeout -k 10 200 python -u tools/bench_kernels.py > gpurun_out/s61/kern_$tt.log 2>&1 || { tail gpurun_out/s61/kern_$tt.log; exit 1; }
  echo "tt=$tt $(grep swiglu_bwd_t gpurun_out/s61/kern_$tt.log)"
done
for tt in 64 128; do
  DTG_SWIGLU_TT=$tt timeout -k 10 300 python -u bench.py > gpurun_out/s61/bench_$tt.log 2>&1 || { tail gpurun_out/s61/bench_$tt.log; exit 1; }
  echo "bench tt=$tt $(tail -1 gpurun_out/s61/bench_$tt.log | cut -c1-200)"
done
