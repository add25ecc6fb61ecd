#!/bin/bash
# Full GPU suite + elastic-recovery demo logs + short bench.
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && OUT=gpurun_out/check3 && mkdir -p $OUT
timeout -k 10 300 python scripts/elastic_demo.py --ranks 3 --out $OUT/elastic_demo > $OUT/elastic_demo.log 2>&1 &&
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 3 --warmup 1 > $OUT/bench.json 2> $OUT/bench.log
echo "exit $?"
