#!/usr/bin/env bash
# r4_s30: TunableOp candidate list (verbose log format) + sustained timing of the committed picks.
set -o pipefail
out=gpurun_out/r4_s30
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/tunableop_sustained.py list --only gu_fwd,o_fwd --out "$out/cands.json" > "$out/list.log" 2>&1 \
    || { tail -30 "$out/list.log"; exit 1; }
tail -5 "$out/list.log"
timeout -k 10 300 python -u tools/tunableop_sustained.py _time --seconds 2 > "$out/committed.log" 2>&1 \
    || { tail -30 "$out/committed.log"; exit 1; }
cat "$out/committed.log" | cut -c1-200
