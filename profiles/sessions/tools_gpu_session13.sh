#!/bin/bash
# Tune the weight-gradient (and forward/dX) GEMMs of Llama-3-8B at 16k tokens with TunableOp.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s13
export TMPDIR=/tmp
timeout -k 10 1000 python tools/tune_gemms.py --which dw --out gpurun_out/s13/tunableop_dw.csv > gpurun_out/s13/tune_dw.log 2>&1
rc=$?; echo "tune dw rc=$rc"; tail -5 gpurun_out/s13/tune_dw.log
exit $rc
