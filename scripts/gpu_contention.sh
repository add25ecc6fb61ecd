#!/bin/bash
# CU reservation for RCCL: probe-kernel launch latency under a CRC burst, then the GPU suite.
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && OUT=gpurun_out/${1:-contention} && mkdir -p $OUT
timeout -k 10 120 bin/contention -trials 40 -reserve 32 > $OUT/contention.jsonl 2>&1 &&
timeout -k 10 120 bin/contention -trials 40 -reserve 64 > $OUT/contention64.jsonl 2>&1 &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
echo "exit $?"
