#!/usr/bin/env bash
# r4_s31: every TunableOp survivor of the 8B step's 11 TN GEMM shapes, timed under sustained load.
set -o pipefail
out=gpurun_out/r4_s31
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/tunableop_sustained.py list --out "$out/cands.json" > "$out/list.log" 2>&1 \
    || { tail -30 "$out/list.log"; exit 1; }
gzip -f "$out/cands.json.log"
timeout -k 10 900 python -u tools/tunableop_sustained.py time --cands "$out/cands.json" --top 9 --seconds 2 \
    --out "$out/sustained.jsonl" > "$out/time.log" 2>&1 || { tail -30 "$out/time.log"; exit 1; }
wc -l "$out/sustained.jsonl"
