#!/bin/bash
# Re-verify the restored tree on a fresh box (GPU tests, smoke, bench) and time every GEMM layout.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s14
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s14/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/s14/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s14/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/s14/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/s14/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/s14/bench.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_gemm_layouts.py > gpurun_out/s14/gemm_layouts_hipblaslt.jsonl 2>&1
rc=$?; echo "layouts rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_gemm_layouts.py --blas rocblas > gpurun_out/s14/gemm_layouts_rocblas.jsonl 2>&1
rc=$?; echo "layouts rocblas rc=$rc"
exit $rc
