#!/bin/bash
# One entry point for every GPU-box recipe (run through gpurun):
#
#   gpurun --timeout 1200 -- bash scripts/gpu.sh <recipe> [out-subdir]
#
# Every GPU step runs under its own `timeout -k`, steps are chained with &&,
# and output goes to gpurun_out/<out-subdir> (default: the recipe name).
# (Rounds 1-4's A/B recipes for kernel variants that no longer exist are in
# the git history; their results stay under profiles/.)
#
# Recipes
#   check      GPU tests, smoke(), 1-GPU headline bench
#   verify     receive-side kernels at the engine's launch size: tests + scripts/verify_bench.py + kernel trace
#   profile    kernel traces of the headline bench and the fp8 --store bf16 receive path
#   pmc        counters of the two verify kernels at the engine's full-batch launch (3 passes)
#   multirank  multi-rank RCCL rehearsal on one GPU (ranks share device 0)
#   shared8    the driver's `bench.py --gpus 8` path at 8 ranks on one GPU (every mode)
#   shared24   the driver's N = 2 and N = 4 scaling points (`bench.py --gpus 2/4`) on one GPU
#   insure     IPC variants, 14-lane rank death at 8 ranks, supervised bench --gpus 8 (+ forced fallback)
#   queues     per-rank rocprofv3 kernel traces of a shared-GPU bench (HW queue ids; QRANKS=8 for 8 ranks)
#   disk       NVMe tier bench + diskspeed
#   fp8        BASELINE #5 at N = 1: full 126 x 3 GiB fp8 preset; --store bf16 subset
#   contention continuous verification at 450 GB/s beside a 64-workgroup copy and RCCL self-P2P
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
RECIPE=${1:-check}
OUT=gpurun_out/${2:-$RECIPE}
mkdir -p "$OUT"
PYTEST="python -u -m pytest -x -v --timeout 300 --timeout-method thread"

case "$RECIPE" in
  check)
    timeout -k 10 900 $PYTEST --durations=30 tests -m gpu > $OUT/pytest_gpu.log 2>&1 &&
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 &&
    timeout -k 10 600 python bench.py --steps 3 --warmup 1 > $OUT/bench.json 2> $OUT/bench.log
    ;;
  verify)
    timeout -k 10 400 $PYTEST tests/test_gpu_kernels.py tests/test_gpu_ops.py > $OUT/pytest.log 2>&1 &&
    timeout -k 10 240 python scripts/verify_bench.py > $OUT/vb.json 2> $OUT/vb.err &&
    timeout -k 10 240 python scripts/verify_bench.py --cus 128 > $OUT/vb_cus128.json 2> $OUT/vb_cus128.err &&
    timeout -k 10 240 python scripts/verify_bench.py --cus 32 > $OUT/vb_cus32.json 2> $OUT/vb_cus32.err &&
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o vb -- \
      python3 scripts/verify_bench.py --reps 20 > $OUT/vb_trace.json 2> $OUT/vb_trace.err
    ;;
  profile)
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/bench -o bench -- \
      python3 bench.py --steps 2 --warmup 1 > $OUT/bench.json 2> $OUT/bench.log &&
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/fp8_bf16 -o fp8b -- \
      python3 bench.py --pack fp8 --store bf16 --layers 20 --layer-mib 3072 --steps 2 --warmup 1 \
      > $OUT/fp8_bf16.json 2> $OUT/fp8_bf16.log
    ;;
  pmc)
    VB="python3 scripts/verify_bench.py --only-full-batch --reps 5"
    timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT \
      SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $OUT/sq -o sq -- $VB \
      > $OUT/sq.json 2> $OUT/sq.err &&
    timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o fetch -- $VB \
      > $OUT/fetch.json 2> $OUT/fetch.err &&
    timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o write -- $VB \
      > $OUT/write.json 2> $OUT/write.err &&
    python3 scripts/pmc_summary.py $OUT/sq $OUT/fetch $OUT/write > $OUT/pmc_summary.md
    ;;
  multirank)
    timeout -k 10 1100 $PYTEST tests/test_gpu_multirank.py > $OUT/pytest.log 2>&1
    ;;
  shared8)
    # SHARED8_SPECS="spec;spec": only these (e.g. a rerun of the last ones)
    rc=0
    SPECS=("1" "1 --seeding uniform" "2 --pull-window 2" "3" "0 --seeding leader" \
           "0 --seeding leader --bcast collective" "1 --pack fp8 --layer-mib 96")
    [ -n "$SHARED8_SPECS" ] && IFS=';' read -r -a SPECS <<< "$SHARED8_SPECS"
    for spec in "${SPECS[@]}"; do
      set -- $spec
      mode=$1; shift
      tag=m${mode}$(echo "$*" | tr -c 'a-z0-9' '_')
      DISSEM_SHARED_GPU=1 timeout -k 10 150 python bench.py --gpus 8 --steps 2 --warmup 1 --layers 16 \
        --layer-mib 64 --chunk-mib 16 --mode "$mode" "$@" > $OUT/bench_$tag.json 2> $OUT/bench_$tag.log || { rc=$?; break; }
    done
    [ $rc -eq 0 ]
    ;;
  shared24)
    DISSEM_SHARED_GPU=1 timeout -k 10 240 python bench.py --gpus 2 --steps 2 --warmup 1 --layers 16 --layer-mib 64 \
      --chunk-mib 16 > $OUT/bench_n2.json 2> $OUT/bench_n2.log &&
    DISSEM_SHARED_GPU=1 timeout -k 10 240 python bench.py --gpus 4 --steps 2 --warmup 1 --layers 16 --layer-mib 64 \
      --chunk-mib 16 > $OUT/bench_n4.json 2> $OUT/bench_n4.log
    ;;
  insure)
    # For the first real 8-GPU run: cross-process IPC variants, the 14-lane
    # rank-death recovery at 8 ranks, bench.py --gpus 8 through the supervisor
    # with the link probe, and a forced first-attempt failure.
    DISSEM_TEST_LOGDIR=$OUT/ipc timeout -k 10 200 $PYTEST tests/test_gpu_ipc.py > $OUT/pytest_ipc.log 2>&1 &&
    DISSEM_FULL_REHEARSAL=1 DISSEM_TEST_LOGDIR=$OUT/death8 timeout -k 10 400 $PYTEST tests/test_gpu_multirank.py \
      -k "rank_death and full" > $OUT/pytest_death8.log 2>&1 &&
    DISSEM_SHARED_GPU=1 timeout -k 10 300 python bench.py --gpus 8 --steps 2 --warmup 1 --layers 16 \
      --layer-mib 64 --chunk-mib 16 --probe-mib 64 > $OUT/bench8_probe.json 2> $OUT/bench8_probe.log &&
    DISSEM_SHARED_GPU=1 timeout -k 10 400 python bench.py --gpus 8 --steps 2 --warmup 1 --layers 16 \
      --layer-mib 64 --chunk-mib 16 --probe-mib 64 --inject fail-attempt=3@0 \
      > $OUT/bench8_fallback.json 2> $OUT/bench8_fallback.log
    ;;
  queues)
    # Plain per-rank processes (no torchrun): rocprofv3 wraps the python program itself.
    # QRANKS ranks (default 3; 8 = the driver's lane count, 14 lanes per rank).
    NR=${QRANKS:-3}
    pids=()
    for r in $(seq 0 $((NR - 1))); do
      DISSEM_SHARED_GPU=1 RANK=$r LOCAL_RANK=0 WORLD_SIZE=$NR MASTER_ADDR=127.0.0.1 MASTER_PORT=29517 \
        timeout -s KILL 300 rocprofv3 --kernel-trace --marker-trace --output-format csv -d $OUT/rank$r -o q -- \
        python3 bench.py --gpus $NR --steps 2 --warmup 1 --layers $((NR * 2)) --layer-mib 64 --chunk-mib 16 \
        > $OUT/rank$r.json 2> $OUT/rank$r.log &
      pids+=($!)
    done
    rc=0
    for p in "${pids[@]}"; do wait $p || rc=$?; done
    [ $rc -eq 0 ] && python3 scripts/queue_summary.py $OUT > $OUT/queues.txt 2>&1
    ;;
  disk)
    # BASELINE config #4 at N = 1, cold: layer files under ./storage (the box's root file system),
    # every file's page-cache pages evicted before every session, O_DIRECT reads counted (the
    # JSON's disk_read_mode / storage_fs / page_cache_resident_max); DISK_LAYERS layers of 1 GiB
    # (80 when the disk holds them - the JSON's layers_fit_on_storage says what does), then
    # bin/diskspeed over ALL files of the same run (O_DIRECT, 4 and 8 readers), evicted again first
    L=${DISK_LAYERS:-72}
    df -hT . > $OUT/df.txt 2>&1; lsblk -o NAME,SIZE,TYPE,ROTA,MOUNTPOINT >> $OUT/df.txt 2>&1
    timeout -k 10 900 python bench.py --tier disk --layers $L --steps 2 --warmup 1 \
      > $OUT/bench_disk.json 2> $OUT/bench_disk.log &&
    DROP="import sys; sys.path.insert(0, '.'); from distributed_llm_dissemination_amd import _core; \
print(max(_core.file_cache_drop(f'storage/layers/0/{l}.layer') for l in range($L)))"
    FILES=$(for l in $(seq 0 $((L - 1))); do echo "-path storage/layers/0/$l.layer"; done)
    python -c "$DROP" > $OUT/cache_drop.txt &&
    timeout -k 10 300 bin/diskspeed $FILES -depth 4 > $OUT/diskspeed_all_d4.log 2>&1 &&
    python -c "$DROP" >> $OUT/cache_drop.txt &&
    timeout -k 10 300 bin/diskspeed $FILES -depth 8 > $OUT/diskspeed_all_d8.log 2>&1 &&
    rm -rf storage
    ;;
  fp8)
    # BASELINE config #5 at N = 1: the full 126 x 3 GiB preset (bf16 sources from an 8-buffer
    # pinned pool), and the --store bf16 receive path on a 20 x 3 GiB subset
    timeout -k 10 900 python bench.py --preset llama405b-fp8 --source-pool 8 --steps 2 --warmup 1 \
      > $OUT/bench_405b_fp8.json 2> $OUT/bench_405b_fp8.log &&
    timeout -k 10 600 python bench.py --pack fp8 --store bf16 --layers 20 --layer-mib 3072 \
      --steps 2 --warmup 1 > $OUT/bench_fp8_store_bf16.json 2> $OUT/bench_fp8_store_bf16.log
    ;;
  contention)
    # continuous verification at the landing rate of 7 links (450 GB/s) beside a 64-workgroup copy
    timeout -k 10 120 bin/contention -cumap > $OUT/cumap.jsonl 2>&1 &&
    timeout -k 10 400 bin/contention -paced 10 -gbps 450 > $OUT/paced.jsonl 2>&1 &&
    timeout -k 10 240 bin/contention -rccl 8 -gbps 450 > $OUT/rccl_paced.jsonl 2> $OUT/rccl_paced.log
    ;;
  *)
    echo "unknown recipe $RECIPE" >&2
    exit 2
    ;;
esac
rc=$?
echo "recipe $RECIPE exit $rc"
exit $rc
