#!/bin/bash
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/prof2
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_engine.py -x -q --timeout 120 > gpurun_out/pytest_gpu2.log 2>&1 &&
timeout -k 10 300 python scripts/kernel_bench.py > gpurun_out/kernel_bench2.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof2 -o pmc_fetch -- python3 scripts/kernel_bench.py > gpurun_out/prof_pmc_fetch.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof2 -o pmc_write -- python3 scripts/kernel_bench.py > gpurun_out/prof_pmc_write.log 2>&1 &&
mkdir -p /tmp/dl_disk && timeout -k 10 900 python bench.py --tier disk --layers 16 --storage /tmp/dl_disk --steps 2 --warmup 1 > gpurun_out/bench_disk.log 2>&1 &&
timeout -k 10 120 bin/diskspeed -path /tmp/dl_disk/layers/0/$(ls /tmp/dl_disk/layers/0 | head -1) > gpurun_out/diskspeed.log 2>&1
