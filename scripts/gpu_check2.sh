#!/bin/bash
# Health check of the tree: GPU tests, smoke(), kernel microbench, short 1-GPU bench.
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/check2
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/check2/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/check2/smoke.log 2>&1 &&
timeout -k 10 300 python scripts/kernel_bench.py > gpurun_out/check2/kernel_bench.json 2> gpurun_out/check2/kernel_bench.log &&
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/check2/bench.json 2> gpurun_out/check2/bench.log
echo "exit $?"
