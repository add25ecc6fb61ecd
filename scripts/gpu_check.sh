#!/bin/bash
# Round-end style GPU check: GPU tests, smoke(), default bench (1 GPU), kernel-trace profile.
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/check
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/check/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/check/smoke.log 2>&1 &&
timeout -k 10 600 python bench.py > gpurun_out/check/bench.json 2> gpurun_out/check/bench.log
echo "exit $?"
