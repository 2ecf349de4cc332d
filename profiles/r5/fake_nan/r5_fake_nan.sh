#!/usr/bin/env bash
# Localise the non-finite values of the DTG_FAKE_WORLD tensor-parallel rehearsal (8B, tp 8).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5_fake_nan}
mkdir -p "$O"
export TMPDIR=/tmp
for lr in 0 3e-5; do
  DTG_FAKE_WORLD=8 timeout -k 10 240 python -u tools/diag_fake_nan.py --tp 8 --steps 14 --lr $lr > "$O/diag_lr$lr.jsonl" 2>&1 \
      || { tail -20 "$O/diag_lr$lr.jsonl"; exit 1; }
  grep '^{' "$O/diag_lr$lr.jsonl" | cut -c1-300
done
