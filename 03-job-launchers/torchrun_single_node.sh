#!/bin/bash
# Single node, one rank per MI355X: rank logs under ../logs, failing rank's
# traceback in ../error.json.
#   ./torchrun_single_node.sh <chapter-dir> <train_llm.py args...>
set -euo pipefail
CHAPTER=${1:?chapter dir}; shift
export TORCHELASTIC_ERROR_FILE=${TORCHELASTIC_ERROR_FILE:-../error.json}
export OMP_NUM_THREADS=${OMP_NUM_THREADS:-1}
export HSA_ENABLE_IPC_MODE_LEGACY=${HSA_ENABLE_IPC_MODE_LEGACY:-0}
python -m torch.distributed.run --standalone --nproc-per-node gpu --redirects 3 --log-dir ../logs \
  "../$CHAPTER/train_llm.py" "$@"
