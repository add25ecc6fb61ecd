#!/bin/bash
# Repeated full CPU-suite runs (`pytest tests -x -q -m "not gpu"`, as the
# driver runs it), each leaving a JUnit XML report and - when it fails - its
# whole output, so a flake is caught by name with its traceback instead of
# guessed at. Optionally beside a scratch tree rebuilding in a loop with
# `make -B -j16` on the same CPUs (LOAD=1).
#
#   bash scripts/determinism_run.sh [runs=5] [workers=0 (serial) | N (pytest -n N)] [dir=profiles/r6_determinism]
#
# Run it from a copy of the tree (TREE=<commit> names it in the summary) when
# the working tree's extension is rebuilt meanwhile.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
RUNS=${1:-5}
WORKERS=${2:-0}
DIR=${3:-profiles/r6_determinism}
mkdir -p "$DIR"
TAG=$([ "$WORKERS" -gt 0 ] && echo "n$WORKERS" || echo serial)
SUMMARY="$DIR/summary_$TAG.txt"
if [ "${LOAD:-0}" = 1 ]; then
  SCRATCH=$(mktemp -d /tmp/dissem_load.XXXXXX)
  cp -r Makefile csrc "$SCRATCH"/ && mkdir -p "$SCRATCH/distributed_llm_dissemination_amd"
  # own process group, so the trap stops the loop and the make it is running
  setsid bash -c "cd '$SCRATCH' && while true; do make -B -j16 > /dev/null 2>&1; done" &
  LOADPID=$!
  trap 'kill -- -$LOADPID 2>/dev/null; wait $LOADPID 2>/dev/null; rm -rf "$SCRATCH"' EXIT
fi
{
  echo "# $RUNS CPU-suite runs ($TAG$([ "${LOAD:-0}" = 1 ] && echo ', beside a looping make -B -j16')), $(nproc) CPUs, $(date -u +%FT%TZ)"
  echo "# tree: ${TREE:-$(git rev-parse --short HEAD)$(git diff --quiet || echo '+dirty')}"
} >> "$SUMMARY"
XDIST=()
[ "$WORKERS" -gt 0 ] && XDIST=(-n "$WORKERS")
# tests/conftest.py runs -m "not gpu" on 4 workers unless told otherwise
[ "$WORKERS" -eq 0 ] && export DISSEM_TEST_SERIAL=1
rc=0
for i in $(seq 1 "$RUNS"); do
  start=$(date +%s)
  LOGF="$DIR/${TAG}_run$i.log"
  timeout 3000 python -m pytest tests/ -x -q -m "not gpu" -p no:cacheprovider "${XDIST[@]}" \
    --junitxml="$DIR/${TAG}_run$i.xml" > "$LOGF" 2>&1
  st=$?
  last=$(tail -1 "$LOGF")
  failed=$(grep -E '^(FAILED|ERROR) ' "$LOGF" | head -5 | tr '\n' ' ')
  echo "run $i: ${last} (load $(cut -d' ' -f1-3 /proc/loadavg), $(($(date +%s) - start)) s, exit $st)${failed:+ -- $failed}" >> "$SUMMARY"
  if [ $st -eq 0 ]; then
    rm -f "$LOGF"  # a pass keeps its XML report only
  else
    rc=1
  fi
done
echo "all runs passed: $([ $rc -eq 0 ] && echo yes || echo NO)" >> "$SUMMARY"
exit $rc
