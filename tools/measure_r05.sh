#!/bin/bash
# Round-5 measurement session (VERDICT r04 items 2, 3 and ADVICE r04 PTRS margins).
#   tools/measure_r05.sh TAG [sweep|strong|ptrs ...]      (default: all)
# sweep:  InvMgmt Backlog step and K=30 rollout at 65 536 / 262 144 / 524 288 /
#         1 048 576 envs: a bench line (HIP-event kernel time), rocprofv3
#         kernel-trace stats and separate FETCH_SIZE / WRITE_SIZE passes each.
#         Past ~256 MiB of state the working set no longer fits the Infinity
#         Cache, so the counters see HBM traffic only.
# strong: the per-rank sizes of configs 4 and 5 under 1->8 strong / weak
#         scaling: Net Backlog 32 768 / 16 384 / 8 192 / 4 096 envs and
#         LostSales 32 768 / 8 192, each with the eager step line, the fused
#         K=30 rollout and the StepGraph replay (bench.py's default regions).
# timing: per-wave timelines of the InvMgmt step (TIMING build) and
#         tools/launch_overlap.py (event vs isolated launch times).
# ptrs:   tools/ptrs_margin.py on the decide (default) and branchy PTRS-stats builds.
# Output under gpurun_out/meas_TAG/.  Stops at the first failing step.
set -u
TAG=${1:-r05}; shift || true
PARTS=${*:-sweep strong ptrs}
OUT=gpurun_out/meas_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
run() {
    echo "+ $*" >&2
    "$@"
    rc=$?
    if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" >&2; exit $rc; fi
}
B="--no-cpu-baseline --no-graph-line"
for part in $PARTS; do
  case $part in
  sweep)
    for n in 65536 262144 524288 1048576; do
      P=$OUT/sweep/n$n
      mkdir -p $P
      run timeout -k 10 180 python bench.py --n-envs $n --steps 400 --warmup 40 $B > $P/bench.json 2>$P/bench.err
      tail -n1 $P/bench.json | cut -c1-160
      S="--n-envs $n --steps 300 --warmup 30 $B --no-rollout-line"
      R="--n-envs $n --mode rollout --steps 600 --warmup 60 $B"
      run timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace -o run -- \
          python bench.py $S > $P/trace.log 2>&1
      run timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace_roll -o run -- \
          python bench.py $R > $P/trace_roll.log 2>&1
      run timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/pmc_fetch -o run -- \
          python bench.py $S > $P/fetch.log 2>&1
      run timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/pmc_write -o run -- \
          python bench.py $S > $P/write.log 2>&1
      run timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/pmc_fetch_roll -o run -- \
          python bench.py $R > $P/fetch_roll.log 2>&1
      run timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/pmc_write_roll -o run -- \
          python bench.py $R > $P/write_roll.log 2>&1
    done ;;
  strong)
    mkdir -p $OUT/strong
    for spec in net_backlog:32768 net_backlog:16384 net_backlog:8192 net_backlog:4096 \
                invmgmt_lostsales:32768 invmgmt_lostsales:8192; do
      w=${spec%%:*}; n=${spec##*:}
      run timeout -k 10 180 python bench.py --workload $w --n-envs $n --steps 2000 --warmup 100 --no-cpu-baseline \
          > $OUT/strong/${w}_$n.json 2>$OUT/strong/${w}_$n.err
      tail -n1 $OUT/strong/${w}_$n.json | cut -c1-160
      run timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/strong/trace_${w}_$n -o run -- \
          python bench.py --workload $w --n-envs $n --steps 1000 --warmup 50 --no-cpu-baseline \
          > $OUT/strong/trace_${w}_$n.log 2>&1
    done ;;
  timing)
    # per-wave timelines of the InvMgmt step (TIMING build): the LostSales
    # 32 768-env shard and the Backlog 65 536 headline, then the event vs
    # isolated-launch comparison of the four step kernels
    mkdir -p $OUT/timing
    export INVSIM_LIB=or-gym-inventory_amd/invsim/_lib/timing/libinvsim_TIMING.so
    run timeout -k 10 120 python tools/timing_im_step.py 32768 lostsales > $OUT/timing/im_step_lostsales_32768.txt 2>&1
    run timeout -k 10 120 python tools/timing_im_step.py 65536 > $OUT/timing/im_step_backlog_65536.txt 2>&1
    unset INVSIM_LIB
    cat $OUT/timing/im_step_lostsales_32768.txt
    run timeout -k 10 300 python tools/launch_overlap.py > $OUT/timing/launch_overlap.txt 2>&1
    cat $OUT/timing/launch_overlap.txt ;;
  ptrs)
    for v in ptrs_stats ptrs_stats_branchy; do
      export INVSIM_LIB=or-gym-inventory_amd/invsim/_lib/debug/libinvsim_$v.so
      run timeout -k 10 300 python tools/ptrs_margin.py > $OUT/ptrs_margin_$v.json 2>$OUT/ptrs_margin_$v.err
      unset INVSIM_LIB
      tail -c 400 $OUT/ptrs_margin_$v.json
    done ;;
  esac
done
echo "measure $TAG done"
