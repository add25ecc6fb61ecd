#!/bin/bash
# One node, N MI355X ranks (one process per GPU) over RCCL/xGMI:
#   scripts/launch_gpus.sh N CONFIG MODE [extra CLI flags...]
# e.g. scripts/launch_gpus.sh 8 conf/llama70b_mode1_random.json 1 --json-summary
set -euo pipefail
N=$1
CONFIG=$2
MODE=$3
shift 3
HERE="$(cd "$(dirname "$0")/.." && pwd)"
export PYTHONPATH="$HERE${PYTHONPATH:+:$PYTHONPATH}"
PORT=$(python3 -c "import socket;s=socket.socket();s.bind(('127.0.0.1',0));print(s.getsockname()[1])")
python3 -m torch.distributed.run --nnodes=1 --nproc-per-node "$N" --master-addr 127.0.0.1 --master-port "$PORT" \
  -m distributed_llm_dissemination_amd -f "$CONFIG" -m "$MODE" --engine rccl "$@"
