# Driver scaling points N = 2 and 4 rehearsed on one GPU (ranks share device 0, RCCL over sockets):
# the fused-kernel tests first, then bench.py --gpus 2/4 through torchrun.
set -o pipefail
OUT=gpurun_out/r2_shared24
mkdir -p $OUT
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "fused" > $OUT/pytest_fused.log 2>&1 || exit 1
for n in 2 4; do
  DISSEM_SHARED_GPU=1 timeout -k 10 240 python bench.py --gpus $n --steps 2 --warmup 1 --layers 16 --layer-mib 64 --chunk-mib 16 > $OUT/bench_n$n.json 2> $OUT/bench_n$n.log || exit 1
done
DISSEM_SHARED_GPU=1 timeout -k 10 240 python bench.py --gpus 2 --steps 2 --warmup 1 --layers 8 --layer-mib 1024 > $OUT/bench_n2_1GiB.json 2> $OUT/bench_n2_1GiB.log
