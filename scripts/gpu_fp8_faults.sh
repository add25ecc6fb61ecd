#!/bin/bash
# GPU validation of the fp8 path + fault handling: GPU tests, kernel microbench
# (incl. fused verify+unpack), headline bench, fp8 bench, kernel-trace profile.
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/fp8
timeout -k 10 600 python -m pytest tests -m gpu -x -q --timeout 300 > gpurun_out/fp8/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python scripts/kernel_bench.py > gpurun_out/fp8/kernel_bench.json 2> gpurun_out/fp8/kernel_bench.err &&
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/fp8/bench_70b.json 2> gpurun_out/fp8/bench_70b.log &&
timeout -k 10 600 python bench.py --steps 2 --warmup 1 --pack fp8 --layers 20 --layer-mib 3072 > gpurun_out/fp8/bench_fp8.json 2> gpurun_out/fp8/bench_fp8.log &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fp8/prof -o kb -- python3 scripts/kernel_bench.py > gpurun_out/fp8/prof.log 2>&1
echo "exit $?"
