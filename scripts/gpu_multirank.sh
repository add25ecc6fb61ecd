#!/bin/bash
# Multi-rank RCCL rehearsal on a one-GPU box: ranks share device 0 (DISSEM_SHARED_GPU, utils/launch.py).
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/multirank
timeout -k 10 900 python -u -m pytest tests/test_gpu_multirank.py -x -v --timeout 300 --timeout-method thread > gpurun_out/multirank/pytest.log 2>&1
echo "exit $?"
