#!/bin/bash
# Run one node (reference: conf/exe.sh). Positional args as in the reference:
#   scripts/run_node.sh ID MODE IS_DISK IS_SETUP [CONFIG] [STORAGE]
# IS_DISK=1 keeps layers as files under STORAGE (default /mnt/ssd); IS_SETUP=1
# first creates the layer files (-l) and exits that step. Page-cache dropping
# (the reference's `echo 1 > /proc/sys/vm/drop_caches`) needs root and is
# skipped otherwise; the GPU engine reads disk layers with O_DIRECT anyway.
set -euo pipefail
ID=$1
MODE=$2
IS_DISK=$3
IS_SETUP=$4
CONFIG=${5:-config.json}
STORAGE=${6:-/mnt/ssd}
HERE="$(cd "$(dirname "$0")/.." && pwd)"
export PYTHONPATH="$HERE${PYTHONPATH:+:$PYTHONPATH}"

SSD_FLAG=()
if [ "$IS_DISK" -eq 1 ]; then
  SSD_FLAG=(-s "$STORAGE")
fi
if [ "$IS_SETUP" -eq 1 ]; then
  python3 -m distributed_llm_dissemination_amd -id "$ID" -f "$CONFIG" "${SSD_FLAG[@]}" -m "$MODE" -l -v
fi
if [ "$(id -u)" -eq 0 ]; then
  sync && echo 1 > /proc/sys/vm/drop_caches || true
fi
exec python3 -m distributed_llm_dissemination_amd -id "$ID" -f "$CONFIG" "${SSD_FLAG[@]}" -m "$MODE" -v \
  2> "log${ID}.jsonl"
