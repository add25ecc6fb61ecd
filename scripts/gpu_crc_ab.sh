#!/bin/bash
# CRC32C kernels: numerics, throughput, kernel trace, LDS/VALU counters.
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && OUT=gpurun_out/${1:-crc} && mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 &&
timeout -k 10 300 python scripts/kernel_bench.py > $OUT/kernel_bench.json 2> $OUT/kernel_bench.log &&
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o kb -- python3 scripts/kernel_bench.py > $OUT/trace.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $OUT/pmc -o lds -- python3 scripts/kernel_bench.py > $OUT/pmc.log 2>&1
echo "exit $?"
