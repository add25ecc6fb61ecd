#!/bin/bash
# Kernel + copy trace of the headline bench (current kernels), and of the fp8 preset subset.
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && OUT=gpurun_out/prof3 && mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/bench -o bench -- python3 bench.py --steps 2 --warmup 1 > $OUT/bench.log 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/fp8 -o fp8 -- python3 bench.py --pack fp8 --layers 20 --layer-mib 3072 --steps 2 --warmup 1 > $OUT/fp8.log 2>&1
echo "exit $?"
