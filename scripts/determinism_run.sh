#!/bin/bash
# N consecutive full CPU-suite runs (`pytest tests -x -q -m "not gpu"`, as the
# driver runs it) while a scratch copy of the tree rebuilds in a loop with
# `make -B -j16` on the same CPUs: the suite must pass every time under load.
#
#   bash scripts/determinism_run.sh [runs=5] [log=profiles/r5_determinism.txt]
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
RUNS=${1:-5}
LOG=${2:-profiles/r5_determinism.txt}
SCRATCH=$(mktemp -d /tmp/dissem_load.XXXXXX)
cp -r Makefile csrc "$SCRATCH"/ && mkdir -p "$SCRATCH/distributed_llm_dissemination_amd"
# own process group, so the trap stops the loop and the make it is running
setsid bash -c "cd '$SCRATCH' && while true; do make -B -j16 > /dev/null 2>&1; done" &
LOADPID=$!
trap 'kill -- -$LOADPID 2>/dev/null; wait $LOADPID 2>/dev/null; rm -rf "$SCRATCH"' EXIT
{
  echo "# $RUNS full CPU-suite runs beside a looping 'make -B -j16' ($(nproc) CPUs), $(date -u +%FT%TZ)"
  echo "# tree: $(git rev-parse --short HEAD)$(git diff --quiet || echo '+dirty')"
} > "$LOG"
rc=0
for i in $(seq 1 "$RUNS"); do
  start=$(date +%s)
  out=$(timeout 3000 python -m pytest tests/ -x -q -m "not gpu" -p no:cacheprovider 2>&1 | tail -1)
  st=$?
  echo "run $i: ${out} (load average $(cut -d' ' -f1-3 /proc/loadavg), $(($(date +%s) - start)) s, exit $st)" >> "$LOG"
  [ $st -eq 0 ] || rc=1
done
echo "all runs passed: $([ $rc -eq 0 ] && echo yes || echo NO)" >> "$LOG"
exit $rc
