#!/bin/bash
# Profiles: kernel throughput, rocprofv3 kernel/copy trace of the 1-GPU bench, disk tier.
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/prof
timeout -k 10 300 python scripts/kernel_bench.py > gpurun_out/kernel_bench.log 2>&1 &&
timeout -k 10 600 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/prof_bench.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE WRITE_SIZE --output-format csv -d gpurun_out/prof -o crcpmc -- python3 scripts/kernel_bench.py > gpurun_out/prof_pmc.log 2>&1 &&
mkdir -p /tmp/dl_disk && timeout -k 10 600 python bench.py --tier disk --layers 16 --storage /tmp/dl_disk --steps 2 --warmup 1 > gpurun_out/bench_disk.log 2>&1 &&
timeout -k 10 120 bin/diskspeed -path /tmp/dl_disk/layers/0/$(ls /tmp/dl_disk/layers/0 | head -1) > gpurun_out/diskspeed.log 2>&1
df -h /tmp . >> gpurun_out/diskspeed.log 2>&1
