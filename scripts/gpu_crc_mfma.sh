#!/bin/bash
# MFMA CRC32C kernel: numerics vs host, A/B throughput vs the nibble-table kernel, kernel trace.
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && OUT=gpurun_out/${1:-crcm} && mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 &&
timeout -k 10 300 python scripts/crc_impl_bench.py > $OUT/crc_impl.json 2> $OUT/crc_impl.log &&
timeout -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o ci -- python3 scripts/crc_impl_bench.py > $OUT/trace.log 2>&1
echo "exit $?"
