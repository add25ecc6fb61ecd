#!/bin/bash
# One entry point for every GPU-box recipe (run through gpurun):
#
#   gpurun --timeout 1200 -- bash scripts/gpu.sh <recipe> [out-subdir]
#
# Every GPU step runs under its own `timeout -k`, steps are chained with &&,
# and output goes to gpurun_out/<out-subdir> (default: the recipe name).
#
# Recipes
#   check      GPU tests, smoke(), 1-GPU headline bench
#   multirank  multi-rank RCCL rehearsal on one GPU (ranks share device 0)
#   shared8    the driver's `bench.py --gpus 8` path at 8 ranks on one GPU (every mode)
#   insure     IPC variants, 14-lane rank death at 8 ranks, supervised bench --gpus 8 (+ forced fallback)
#   init       parallel vs split lane-communicator set-up at 8 shared ranks; rank-death re-form
#   r3rehearse host-share (config #2), disk tier + node NVMe budget (config #4) at 8 shared ranks; N = 1 A/Bs
#   r3kernels  fused verify+unpack store A/B + counters, copy bandwidth beside CRC, NUMA A/B
#   r4kernels  walk access patterns, kernel numerics, fused store A/B (walk vs one segment per wave) + counters
#   r4contention  continuous CRC verification at 450 GB/s beside a 64-workgroup copy, per CRC grid cap
#   multihost  8 shared ranks rehearsed as 2 hosts x 4 GPUs: host-aware lanes, hierarchical vs flat modes 1/0, modes 2/3
#   shared24   the driver's N = 2 and N = 4 scaling points (`bench.py --gpus 2/4`) on one GPU
#   queues     per-rank rocprofv3 kernel traces of a shared-GPU bench (HW queue ids; QRANKS=8 for 8 ranks)
#   crc        CRC32C kernels: numerics, A/B throughput, kernel trace, LDS/VALU counters
#   profile    kernel trace of the headline bench and the fp8 subset
#   disk       NVMe tier bench + diskspeed
#   fp8        BASELINE #5 at N = 1: full 126 x 3 GiB fp8 preset; --store bf16 subset
#   crcpmc     SQ issue/wait counters + fetch of the CRC segment kernel
#   contention probe-kernel launch delay under a CRC burst (CU reservation)
#   poolshare  fp8 8 x 3 GiB staging with 0 / 2 / 8 pooled source buffers (shared vs distinct sources)
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
  multirank)
    timeout -k 10 1100 $PYTEST tests/test_gpu_multirank.py > $OUT/pytest.log 2>&1
    ;;
  shared8)
    rc=0
    for spec in "1" "1 --seeding uniform" "2 --pull-window 2" "3" "0 --seeding leader" \
                "0 --seeding leader --bcast collective" "1 --pack fp8 --layer-mib 96"; do
      set -- $spec
      mode=$1; shift
      tag=m${mode}$(echo "$*" | tr -c 'a-z0-9' '_')
      DISSEM_SHARED_GPU=1 timeout -k 10 150 python bench.py --gpus 8 --steps 2 --warmup 1 --layers 16 \
        --layer-mib 64 --chunk-mib 16 --mode "$mode" "$@" > $OUT/bench_$tag.json 2> $OUT/bench_$tag.log || { rc=$?; break; }
    done
    [ $rc -eq 0 ]
    ;;
  insure)
    # Round-3 insurance for the first real 8-GPU run: cross-process IPC variants,
    # the 14-lane rank-death recovery at 8 ranks, bench.py --gpus 8 through the
    # supervisor with the link probe, and a forced first-attempt failure.
    DISSEM_TEST_LOGDIR=$OUT/ipc timeout -k 10 200 $PYTEST tests/test_gpu_ipc.py > $OUT/pytest_ipc.log 2>&1 &&
    DISSEM_FULL_REHEARSAL=1 DISSEM_TEST_LOGDIR=$OUT/death8 timeout -k 10 400 $PYTEST tests/test_gpu_multirank.py \
      -k "rank_death and full" > $OUT/pytest_death8.log 2>&1 &&
    DISSEM_SHARED_GPU=1 timeout -k 10 300 python bench.py --gpus 8 --steps 2 --warmup 1 --layers 16 \
      --layer-mib 64 --chunk-mib 16 --probe-mib 64 > $OUT/bench8_probe.json 2> $OUT/bench8_probe.log &&
    DISSEM_SHARED_GPU=1 timeout -k 10 400 python bench.py --gpus 8 --steps 2 --warmup 1 --layers 16 \
      --layer-mib 64 --chunk-mib 16 --probe-mib 64 --inject fail-attempt=3@0 \
      > $OUT/bench8_fallback.json 2> $OUT/bench8_fallback.log &&
    timeout -k 10 300 python bench.py --steps 3 --warmup 1 > $OUT/bench1.json 2> $OUT/bench1.log
    ;;
  init)
    # lane communicator set-up: parallel (one id per lane, one group) vs split, at 8 shared ranks;
    # the 14-lane rank-death re-form with the parallel init
    for ci in parallel split; do
      DISSEM_SHARED_GPU=1 timeout -k 10 300 python bench.py --gpus 8 --steps 1 --warmup 1 --layers 16 \
        --layer-mib 64 --chunk-mib 16 --probe-mib 16 --comm-init $ci --no-fallback \
        > $OUT/bench8_$ci.json 2> $OUT/bench8_$ci.log || exit 1
    done
    DISSEM_FULL_REHEARSAL=1 DISSEM_TEST_LOGDIR=$OUT/death8 timeout -k 10 400 $PYTEST tests/test_gpu_multirank.py \
      -k "rank_death" > $OUT/pytest_death.log 2>&1
    ;;
  cvt)
    timeout -k 10 60 bin/cvtprobe > $OUT/cvtprobe.jsonl 2>&1
    ;;
  initdbg)
    # RCCL's own init timing breakdown (NCCL_DEBUG=INFO, INIT) for both lane set-ups at 8 shared ranks
    for ci in parallel split; do
      NCCL_DEBUG=INFO NCCL_DEBUG_SUBSYS=INIT DISSEM_SHARED_GPU=1 timeout -k 10 300 python bench.py --gpus 8 \
        --steps 1 --warmup 0 --layers 8 --layer-mib 16 --chunk-mib 16 --probe-mib 0 --comm-init $ci --no-fallback \
        > $OUT/bench8_$ci.json 2> $OUT/bench8_$ci.log || exit 1
      grep -E "Init timings|Init COMPLETE|communicators ready" $OUT/bench8_$ci.log > $OUT/init_$ci.txt || true
    done
    ;;
  init2)
    # lane-communicator set-up with RCCL's ring/tree connections deferred to first use
    # (NCCL_RUNTIME_CONNECT=1; the lanes' P2P connections are still made eagerly by connect_all)
    for ci in parallel split; do
      NCCL_RUNTIME_CONNECT=1 NCCL_DEBUG=INFO NCCL_DEBUG_SUBSYS=INIT DISSEM_SHARED_GPU=1 timeout -k 10 300 \
        python bench.py --gpus 8 --steps 1 --warmup 0 --layers 8 --layer-mib 16 --chunk-mib 16 --probe-mib 0 \
        --comm-init $ci --no-fallback > $OUT/bench8_rc_$ci.json 2> $OUT/bench8_rc_$ci.log || exit 1
      grep -E "Init timings" $OUT/bench8_rc_$ci.log > $OUT/init_rc_$ci.txt || true
    done
    NCCL_RUNTIME_CONNECT=1 DISSEM_SHARED_GPU=1 timeout -k 10 300 python bench.py --gpus 8 --steps 2 --warmup 1 \
      --layers 8 --layer-mib 16 --chunk-mib 16 --mode 0 --seeding leader --bcast collective \
      > $OUT/bench8_rc_bcast.json 2> $OUT/bench8_rc_bcast.log
    ;;
  r3rehearse)
    # round-3 paths at 8 shared ranks and N = 1: config #2 with --host-share, config #4 (disk tier, node
    # NVMe budget) in modes 1 and 3, the supervised default bench; N = 1 staging from shm vs hipHostMalloc
    mkdir -p /tmp/dld_disk8 &&
    DISSEM_SHARED_GPU=1 timeout -k 10 300 python bench.py --gpus 8 --steps 2 --warmup 1 --layers 16 --layer-mib 64 \
      --chunk-mib 16 --mode 0 --seeding leader --host-share --probe-mib 16 > $OUT/b8_m0_hostshare.json 2> $OUT/b8_m0_hostshare.log &&
    DISSEM_SHARED_GPU=1 timeout -k 10 300 python bench.py --gpus 8 --steps 2 --warmup 1 --layers 16 --layer-mib 64 \
      --chunk-mib 16 --tier disk --storage /tmp/dld_disk8 --probe-mib 16 > $OUT/b8_disk_m1.json 2> $OUT/b8_disk_m1.log &&
    DISSEM_SHARED_GPU=1 timeout -k 10 300 python bench.py --gpus 8 --steps 2 --warmup 1 --layers 16 --layer-mib 64 \
      --chunk-mib 16 --tier disk --storage /tmp/dld_disk8 --mode 3 --probe-mib 16 > $OUT/b8_disk_m3.json 2> $OUT/b8_disk_m3.log &&
    DISSEM_SHARED_GPU=1 timeout -k 10 300 python bench.py --gpus 8 --steps 2 --warmup 1 --layers 16 --layer-mib 64 \
      --chunk-mib 16 --probe-mib 16 > $OUT/b8_m1.json 2> $OUT/b8_m1.log &&
    timeout -k 10 300 python bench.py --steps 3 --warmup 1 > $OUT/b1.json 2> $OUT/b1.log &&
    timeout -k 10 300 python bench.py --steps 3 --warmup 1 --host-share > $OUT/b1_hostshare.json 2> $OUT/b1_hostshare.log &&
    timeout -k 10 600 python bench.py --steps 2 --warmup 1 --tier disk --layers 16 --storage /tmp/dld_disk8 \
      > $OUT/b1_disk.json 2> $OUT/b1_disk.log
    ;;
  r3kernels)
    # fused fp8 verify+unpack store-path A/B (numerics, timing, counters), copy bandwidth beside
    # CRC bursts (bin/contention), and the NUMA-binding A/B (3 x 2 interleaved arms, 5 steps each)
    timeout -k 10 300 $PYTEST tests/test_gpu_kernels.py -k fused > $OUT/pytest_fused.log 2>&1 &&
    timeout -k 10 120 python scripts/fused_ab.py > $OUT/fused_ab.json 2> $OUT/fused_ab.log || exit 1
    timeout -s KILL 60 rocprofv3 -L > $OUT/counters_list.txt 2>&1
    for st in 0 1; do
      timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS \
        SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_INSTS_VALU --output-format csv -d $OUT/pmc_sq_$st -o sq -- \
        python3 scripts/fused_ab.py --store $st --reps 5 > $OUT/pmc_sq_$st.log 2>&1 || exit 1
      timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE TA_BUSY_avr TD_BUSY_avr --output-format csv -d $OUT/pmc_mem_$st \
        -o mem -- python3 scripts/fused_ab.py --store $st --reps 5 > $OUT/pmc_mem_$st.log 2>&1 ||
        { rc=$?; [ $rc -ge 124 ] && exit 1; }  # an unknown counter name fails fast; a kill ends the recipe
    done
    timeout -k 10 180 bin/contention -trials 30 -reserve 32 > $OUT/contention.jsonl 2>&1 || exit 1
    for i in 1 2 3; do
      timeout -k 10 200 python bench.py --steps 5 --warmup 1 > $OUT/numa_bound_$i.json 2> $OUT/numa_bound_$i.log &&
      DISSEM_NUMA_BIND=0 timeout -k 10 200 python bench.py --steps 5 --warmup 1 > $OUT/numa_off_$i.json \
        2> $OUT/numa_off_$i.log || exit 1
    done
    DISSEM_SHARED_GPU=1 timeout -k 10 300 python bench.py --gpus 8 --steps 2 --warmup 1 --layers 16 --layer-mib 128 \
      --chunk-mib 16 --mode 0 --seeding leader --host-share --probe-mib 16 > $OUT/b8_m0_hostshare.json \
      2> $OUT/b8_m0_hostshare.log
    ;;
  r4kernels)
    # round 4: walk access patterns (bin/walkprobe), CRC/fused numerics with the new fold constants,
    # fused store A/B (persistent walk vs one segment per wave) at 512 MiB and 4 GiB, counters of both
    timeout -k 10 120 bin/walkprobe 512 20 > $OUT/walk512.jsonl 2>&1 &&
    timeout -k 10 600 $PYTEST tests/test_gpu_kernels.py > $OUT/pytest_kernels.log 2>&1 &&
    timeout -k 10 120 python scripts/fused_ab.py > $OUT/fused_ab.json 2> $OUT/fused_ab.log &&
    timeout -k 10 200 python scripts/fused_ab.py --src-mib 4096 --reps 5 --store 1 5 7 9 > $OUT/fused_ab_4g.json \
      2> $OUT/fused_ab_4g.log || exit 1
    for st in ${PMC_STORES:-1 7}; do
      timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS \
        SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_INSTS_VALU --output-format csv -d $OUT/pmc_sq_$st -o sq -- \
        python3 scripts/fused_ab.py --store $st --reps 5 > $OUT/pmc_sq_$st.log 2>&1 || exit 1
      timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE TA_BUSY_avr TD_BUSY_avr --output-format csv -d $OUT/pmc_mem_$st \
        -o mem -- python3 scripts/fused_ab.py --store $st --reps 5 > $OUT/pmc_mem_$st.log 2>&1 || exit 1
    done
    ;;
  r4contention)
    # continuous verification at the landing rate of 7 links (450 GB/s) beside a 64-workgroup copy, per CRC grid cap
    timeout -k 10 120 bin/contention -cumap > $OUT/cumap.jsonl 2>&1 &&
    timeout -k 10 400 bin/contention -paced 10 -gbps 450 > $OUT/paced.jsonl 2>&1 &&
    timeout -k 10 240 bin/contention -rccl 8 -gbps 450 > $OUT/rccl_paced.jsonl 2> $OUT/rccl_paced.log
    ;;
  r4sweep)
    # fused store 7/8/9 against the source size (tail of the one-segment-per-wave grid), then the
    # paced contention run with CU-partitioned verify
    timeout -k 10 600 $PYTEST tests/test_gpu_kernels.py tests/test_gpu_ops.py > $OUT/pytest_kernels.log 2>&1 || exit 1
    for mib in 448 480 496 504 512 520 528 544 576; do
      timeout -k 10 60 python scripts/fused_ab.py --src-mib $mib --reps 10 --store 7 8 9 10 > $OUT/sweep_$mib.json \
        2> $OUT/sweep_$mib.log || exit 1
    done
    timeout -k 10 400 bin/contention -paced 10 -gbps 450 > $OUT/paced.jsonl 2>&1
    ;;
  r4trace)
    # fused store 7 against size under a kernel trace: main kernel vs fold durations (fixed per-call cost)
    for mib in 64 128 256 512 1024 2048; do
      timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_$mib -o kt -- \
        python3 scripts/fused_ab.py --src-mib $mib --reps 10 --store 7 8 10 > $OUT/kt_$mib.json 2> $OUT/kt_$mib.log || exit 1
    done
    ;;
  r4vcus)
    # A/B of the verify CU partition at 8 shared ranks, same box, interleaved
    rc=0
    for spec in "1 0" "1 32" "2 0" "2 32" "1 0" "1 32" "2 0" "2 32"; do
      set -- $spec
      DISSEM_SHARED_GPU=1 timeout -k 10 150 python bench.py --gpus 8 --steps 2 --warmup 1 --layers 16 \
        --layer-mib 64 --chunk-mib 16 --mode $1 --verify-cus $2 > $OUT/b_m$1_v$2_$RANDOM.json 2> $OUT/b_m$1_v$2.log \
        || { rc=$?; break; }
    done
    [ $rc -eq 0 ]
    ;;
  r4nt)
    # nontemporal stores: store 7 (staged NT) vs 13 (temporal) vs 9, plain pack/unpack NT; numerics, sizes, trace
    timeout -k 10 600 $PYTEST tests/test_gpu_kernels.py tests/test_gpu_ops.py > $OUT/pytest_kernels.log 2>&1 &&
    timeout -k 10 300 python scripts/kernel_bench.py > $OUT/kernel_bench.json 2> $OUT/kernel_bench.log || exit 1
    for mib in 64 512 4096; do
      timeout -k 10 200 python scripts/fused_ab.py --src-mib $mib --reps 10 --store 7 13 9 7 13 > $OUT/ab_$mib.json \
        2> $OUT/ab_$mib.log || exit 1
    done
    for mib in 64 512 2048; do
      timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_$mib -o kt -- \
        python3 scripts/fused_ab.py --src-mib $mib --reps 10 --store 7 8 > $OUT/kt_$mib.json 2> $OUT/kt_$mib.log || exit 1
    done
    ;;
  r4validate)
    # fused kernel numerics (kernel + ops + engine GPU tests), A/B at 64 / 512 / 4096 MiB, all stores, trace at 512 MiB
    timeout -k 10 600 $PYTEST tests/test_gpu_kernels.py tests/test_gpu_ops.py > $OUT/pytest_kernels.log 2>&1 &&
    timeout -k 10 600 $PYTEST tests/test_gpu_engine.py > $OUT/pytest_engine.log 2>&1 || exit 1
    for mib in 64 512 4096; do
      timeout -k 10 200 python scripts/fused_ab.py --src-mib $mib --reps 20 --store 7 13 7 > $OUT/ab_$mib.json \
        2> $OUT/ab_$mib.log || exit 1
    done
    timeout -k 10 120 python scripts/fused_ab.py > $OUT/fused_ab.json 2> $OUT/fused_ab.log &&
    timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_512 -o kt -- \
      python3 scripts/fused_ab.py --src-mib 512 --reps 10 --store 7 > $OUT/kt_512.json 2> $OUT/kt_512.log
    ;;
  r3mx)
    # power-of-two (E8M0-valued) fp8 scales: unpack via v_cvt_scalef32_pk_bf16_fp8; numerics + fused A/B + counters
    timeout -k 10 400 $PYTEST tests/test_gpu_kernels.py tests/test_gpu_ops.py tests/test_gpu_engine.py -k "fp8 or fused" \
      > $OUT/pytest_fp8.log 2>&1 &&
    timeout -k 10 120 python scripts/fused_ab.py > $OUT/fused_ab.json 2> $OUT/fused_ab.log || exit 1
    for st in 0 1; do
      timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS \
        SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_INSTS_VALU --output-format csv -d $OUT/pmc_sq_$st -o sq -- \
        python3 scripts/fused_ab.py --store $st --reps 5 > $OUT/pmc_sq_$st.log 2>&1 || exit 1
    done
    timeout -k 10 600 python bench.py --pack fp8 --store bf16 --layers 20 --layer-mib 3072 \
      --steps 2 --warmup 1 > $OUT/bench_fp8_store_bf16.json 2> $OUT/bench_fp8_store_bf16.log
    ;;
  r3nocrc)
    # fused verify+unpack with and without its CRC math (store 3/4 = 1/0 minus CRC), CRC-only pass, counters
    timeout -k 10 120 python scripts/fused_ab.py > $OUT/fused_ab.json 2> $OUT/fused_ab.log || exit 1
    for st in 1 3; do
      timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS \
        SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU --output-format csv -d $OUT/pmc_sq_$st -o sq -- \
        python3 scripts/fused_ab.py --store $st --reps 5 > $OUT/pmc_sq_$st.log 2>&1 || exit 1
      timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE TA_BUSY_avr TD_BUSY_avr --output-format csv \
        -d $OUT/pmc_mem_$st -o mem -- python3 scripts/fused_ab.py --store $st --reps 5 > $OUT/pmc_mem_$st.log 2>&1 || exit 1
    done
    ;;
  r3tail)
    # segment rounds: 512 MiB = 16896 segments = 4.125 rounds of 4096 waves; 4 GiB = 33 whole rounds
    timeout -k 10 120 python scripts/fused_ab.py --store 1 3 > $OUT/ab_512.json 2> $OUT/ab_512.log &&
    timeout -k 10 120 python scripts/fused_ab.py --store 1 3 --max-blocks 212 > $OUT/ab_512_mb212.json 2> $OUT/ab_512_mb212.log &&
    timeout -k 10 200 python scripts/fused_ab.py --store 1 3 --src-mib 4096 --reps 5 > $OUT/ab_4096.json 2> $OUT/ab_4096.log
    ;;
  r3tail2)
    # balanced segment rounds by default (seg_grid): fused A/B at 512 MiB and 4 GiB, CRC-only, kernel bench, tests
    timeout -k 10 300 $PYTEST tests/test_gpu_kernels.py -k "crc or fused" > $OUT/pytest.log 2>&1 &&
    timeout -k 10 120 python scripts/fused_ab.py > $OUT/ab_512.json 2> $OUT/ab_512.log &&
    timeout -k 10 200 python scripts/fused_ab.py --store 1 3 --src-mib 4096 --reps 5 > $OUT/ab_4096.json 2> $OUT/ab_4096.log &&
    timeout -k 10 200 python scripts/kernel_bench.py > $OUT/kernel_bench.json 2> $OUT/kernel_bench.log
    ;;
  r3fused2)
    # swizzled LDS staging slot (store=1) vs direct stores, counters; NUMA: GPU's node vs the other node
    timeout -k 10 300 $PYTEST tests/test_gpu_kernels.py -k fused > $OUT/pytest_fused.log 2>&1 &&
    timeout -k 10 120 python scripts/fused_ab.py > $OUT/fused_ab.json 2> $OUT/fused_ab.log || exit 1
    for st in 0 1 2; do
      timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS \
        SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_INSTS_VALU --output-format csv -d $OUT/pmc_sq_$st -o sq -- \
        python3 scripts/fused_ab.py --store $st --reps 5 > $OUT/pmc_sq_$st.log 2>&1 || exit 1
      timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE TA_BUSY_avr TD_BUSY_avr --output-format csv \
        -d $OUT/pmc_mem_$st -o mem -- python3 scripts/fused_ab.py --store $st --reps 5 > $OUT/pmc_mem_$st.log 2>&1 || exit 1
    done
    for i in 1 2; do
      DISSEM_NUMA_NODE=0 timeout -k 10 200 python bench.py --steps 5 --warmup 1 > $OUT/numa_node0_$i.json \
        2> $OUT/numa_node0_$i.log &&
      DISSEM_NUMA_NODE=1 timeout -k 10 200 python bench.py --steps 5 --warmup 1 > $OUT/numa_node1_$i.json \
        2> $OUT/numa_node1_$i.log || exit 1
    done
    ;;
  multihost)
    # 8 ranks on one GPU rehearsed as 2 hosts x 4 GPUs (DISSEM_FAKE_HOSTS=2): host-aware comm lanes
    # (14: 6 per host mesh + 8 across) and the hierarchical mode-1 plan over real RCCL; then the flat plan
    rc=0
    for spec in "1" "1 --no-hierarchical" "0 --seeding leader" "0 --seeding leader --no-hierarchical" "2" "3"; do
      set -- $spec
      mode=$1; shift
      tag=m${mode}$(echo "$*" | tr -c 'a-z0-9' '_')
      DISSEM_SHARED_GPU=1 DISSEM_FAKE_HOSTS=2 timeout -k 10 240 python bench.py --gpus 8 --steps 2 --warmup 1 \
        --layers 16 --layer-mib 64 --chunk-mib 16 --mode "$mode" "$@" > $OUT/bench_$tag.json 2> $OUT/bench_$tag.log || { rc=$?; break; }
    done
    # the one-host headline path on the same tree (lane map unchanged at N = 8)
    [ $rc -eq 0 ] && DISSEM_SHARED_GPU=1 timeout -k 10 240 python bench.py --gpus 8 --steps 2 --warmup 1 --layers 16 \
        --layer-mib 64 --chunk-mib 16 --mode 1 > $OUT/bench_onehost_m1.json 2> $OUT/bench_onehost_m1.log || rc=$?
    [ $rc -eq 0 ]
    ;;
  shared24)
    timeout -k 10 200 $PYTEST tests/test_gpu_kernels.py -k fused > $OUT/pytest_fused.log 2>&1 &&
    DISSEM_SHARED_GPU=1 timeout -k 10 240 python bench.py --gpus 2 --steps 2 --warmup 1 --layers 16 --layer-mib 64 \
      --chunk-mib 16 > $OUT/bench_n2.json 2> $OUT/bench_n2.log &&
    DISSEM_SHARED_GPU=1 timeout -k 10 240 python bench.py --gpus 4 --steps 2 --warmup 1 --layers 16 --layer-mib 64 \
      --chunk-mib 16 > $OUT/bench_n4.json 2> $OUT/bench_n4.log &&
    DISSEM_SHARED_GPU=1 timeout -k 10 240 python bench.py --gpus 2 --steps 2 --warmup 1 --layers 8 --layer-mib 1024 \
      > $OUT/bench_n2_1GiB.json 2> $OUT/bench_n2_1GiB.log
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
  crc)
    timeout -k 10 300 $PYTEST tests/test_gpu_kernels.py > $OUT/pytest.log 2>&1 &&
    timeout -k 10 300 python scripts/kernel_bench.py > $OUT/kernel_bench.json 2> $OUT/kernel_bench.log &&
    timeout -k 10 300 python scripts/crc_impl_bench.py > $OUT/crc_impl.json 2> $OUT/crc_impl.log &&
    timeout -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o ci -- \
      python3 scripts/crc_impl_bench.py > $OUT/trace.log 2>&1 &&
    timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU \
      SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $OUT/pmc -o lds -- python3 scripts/kernel_bench.py \
      > $OUT/pmc.log 2>&1
    ;;
  profile)
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/bench -o bench -- \
      python3 bench.py --steps 2 --warmup 1 > $OUT/bench.log 2>&1 &&
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/fp8 -o fp8 -- \
      python3 bench.py --pack fp8 --layers 20 --layer-mib 3072 --steps 2 --warmup 1 > $OUT/fp8.log 2>&1 &&
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/fp8_bf16 -o fp8b -- \
      python3 bench.py --pack fp8 --store bf16 --layers 20 --layer-mib 3072 --steps 2 --warmup 1 > $OUT/fp8_bf16.log 2>&1
    ;;
  disk)
    mkdir -p /tmp/dl_disk &&
    timeout -k 10 900 python bench.py --tier disk --layers 16 --storage /tmp/dl_disk --steps 2 --warmup 1 \
      > $OUT/bench_disk.json 2> $OUT/bench_disk.log &&
    timeout -k 10 120 bin/diskspeed -path /tmp/dl_disk/layers/0/0.layer > $OUT/diskspeed.log 2>&1
    ;;
  fp8)
    # BASELINE config #5 at N = 1: the full 126 x 3 GiB preset (bf16 sources from an 8-buffer
    # pinned pool), and the --store bf16 receive path on a 20 x 3 GiB subset
    timeout -k 10 900 python bench.py --preset llama405b-fp8 --source-pool 8 --steps 2 --warmup 1 \
      > $OUT/bench_405b_fp8.json 2> $OUT/bench_405b_fp8.log &&
    timeout -k 10 600 python bench.py --pack fp8 --store bf16 --layers 20 --layer-mib 3072 \
      --steps 2 --warmup 1 > $OUT/bench_fp8_store_bf16.json 2> $OUT/bench_fp8_store_bf16.log
    ;;
  storeprof)
    # kernel trace of the --store bf16 receive path (fused verify+unpack per staged chunk)
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o st -- \
      python3 bench.py --pack fp8 --store bf16 --layers 8 --layer-mib 3072 --steps 1 --warmup 1 \
      > $OUT/bench.log 2>&1 &&
    timeout -k 10 300 python scripts/crc_impl_bench.py --quick > $OUT/crc_quick.json 2> $OUT/crc_quick.log
    ;;
  crcpmc)
    # issue/wait breakdown of the CRC kernels (one counter pass, 8 SQ counters)
    timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
      SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS --output-format csv \
      -d $OUT/sq -o sq -- python3 scripts/crc_impl_bench.py --quick > $OUT/sq.log 2>&1 &&
    timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD --output-format csv \
      -d $OUT/fetch -o fetch -- python3 scripts/crc_impl_bench.py --quick > $OUT/fetch.log 2>&1
    ;;
  poolshare)
    rc=0
    # POOL_LAYERS (default 8) layers; POOLS: the pool sizes to run in order (default 0 2 8 2 0)
    L=${POOL_LAYERS:-8}
    for p in ${POOLS:-0 2 8 2 0}; do
      timeout -k 10 150 python bench.py --pack fp8 --layers $L --layer-mib 3072 --source-pool $p --steps 3 --warmup 1 \
        > $OUT/L${L}_pool$p.json 2>> $OUT/L${L}_pool$p.log || { rc=$?; break; }
      python3 -c "import json,sys; print('layers', sys.argv[3], 'pool', sys.argv[1], json.load(open(sys.argv[2]))['ms_per_step'])" \
        $p $OUT/L${L}_pool$p.json $L >> $OUT/summary.txt
    done
    [ $rc -eq 0 ]
    ;;
  contention)
    timeout -k 10 120 bin/contention -trials 40 -reserve 32 > $OUT/contention.jsonl 2>&1 &&
    timeout -k 10 120 bin/contention -trials 40 -reserve 64 > $OUT/contention64.jsonl 2>&1
    ;;
  *)
    echo "unknown recipe $RECIPE" >&2
    exit 2
    ;;
esac
rc=$?
echo "recipe $RECIPE exit $rc"
exit $rc
