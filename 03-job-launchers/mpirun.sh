#!/bin/bash
# OpenMPI launcher: mpirun starts every rank directly; dtg.utils.dist reads
# OMPI_COMM_WORLD_RANK/SIZE/LOCAL_RANK, so the training scripts need no code change.
#   ./mpirun.sh host1:8,host2:8 <experiment-name> [chapter-dir] [args...]
set -euo pipefail
HOSTS=${1:?host1:slots,host2:slots}; EXP=${2:?experiment}; CHAPTER=${3:-02-distributed-data-parallel}
shift 3 || shift $#
MASTER=${HOSTS%%:*}
NP=$(echo "$HOSTS" | tr ',' '\n' | awk -F: '{s+=$2} END {print s}')
mpirun -np "$NP" -H "$HOSTS" -bind-to none -map-by slot \
  -x MASTER_ADDR="$MASTER" -x MASTER_PORT=5001 -x OMP_NUM_THREADS=1 -x HSA_ENABLE_IPC_MODE_LEGACY=0 -x PATH -x LD_LIBRARY_PATH \
  python "../$CHAPTER/train_llm.py" --experiment-name "$EXP" "$@"
