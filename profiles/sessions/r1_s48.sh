#!/bin/bash
# Sustained-load (power-limited) timing of every hipBLASLt solution for the biggest 8B GEMMs.
mkdir -p gpurun_out/s48
( while true; do echo "[s48] alive $(date +%T)"; sleep 30; done ) & HB=$!
trap 'kill $HB' EXIT
for spec in tn_28672_16384_4096_ld_4096_4096_28672 tn_4096_16384_28672_ld_28672_28672_4096 tn_4096_28672_16384_ld_16384_16384_4096 tn_4096_16384_14336_ld_14336_14336_4096; do
  timeout -k 10 300 build/gemm_sustained $spec 0.4 12 >> gpurun_out/s48/sustained.jsonl 2>> gpurun_out/s48/sustained.err
  rc=$?; echo "$spec rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
