#!/bin/bash
# GPU validation pass: kernel numerics, engine sessions, smoke, 1-GPU bench + profile.
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -v --timeout 240 > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py --layers 8 --layer-mib 256 --steps 3 --warmup 1 > gpurun_out/bench_small.log 2>&1 &&
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/bench_full.log 2>&1
