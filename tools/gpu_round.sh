#!/bin/bash
# One GPU session for a round: GPU tests, bench lines for every workload
# (step + rollout), rocprofv3 kernel-trace stats and separate FETCH_SIZE /
# WRITE_SIZE passes per workload and mode, plus SQ counter passes for the
# Newsvendor step and rollout kernels.  Everything lands in
# gpurun_out/round_TAG/.  Stops at the first failing step (no GPU work after a
# fault/timeout).
#   tools/gpu_round.sh TAG [tests|bench|prof|trace3|sq ...]   (default: all)
set -u
TAG=${1:-r01}; shift || true
PARTS=${*:-tests bench prof trace3 sq}
OUT=gpurun_out/round_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
run() {
    echo "+ $*" >&2
    "$@"
    rc=$?
    if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" >&2; exit $rc; fi
}
WLS=${WLS:-"invmgmt_backlog invmgmt_lostsales newsvendor net_backlog"}
# --no-config-lines: the default workload's line would also time configs 2, 4, 5 in the
# same process, and their kernels would enter the traces and counter passes
B="--no-cpu-baseline --no-rollout-line --no-graph-line --no-config-lines"
for part in $PARTS; do
  case $part in
  tests)
    run timeout -k 10 480 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
    tail -2 $OUT/pytest_gpu.log ;;
  bench)
    run timeout -k 10 180 python bench.py > $OUT/bench_default.log 2>&1
    tail -1 $OUT/bench_default.log | cut -c1-300
    for w in $WLS; do
      run timeout -k 10 120 python bench.py --workload $w $B > $OUT/bench_${w}_step.log 2>&1
      run timeout -k 10 120 python bench.py --workload $w --mode rollout --steps 1200 $B \
          > $OUT/bench_${w}_rollout.log 2>&1
      run timeout -k 10 120 python bench.py --workload $w --mode policy --steps 1200 $B \
          > $OUT/bench_${w}_policy.log 2>&1
      tail -n1 $OUT/bench_${w}_step.log | cut -c1-200
    done ;;
  prof)
    for w in $WLS; do
      P=$OUT/prof_$w
      run timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace -o run -- \
          python bench.py --workload $w --steps 1000 --warmup 50 $B > $P.trace.log 2>&1
      run timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace_roll -o run -- \
          python bench.py --workload $w --mode rollout --steps 600 --warmup 60 $B > $P.trace_roll.log 2>&1
      run timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/pmc_fetch -o run -- \
          python bench.py --workload $w --steps 200 --warmup 20 $B > $P.fetch.log 2>&1
      run timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/pmc_write -o run -- \
          python bench.py --workload $w --steps 200 --warmup 20 $B > $P.write.log 2>&1
      run timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/pmc_fetch_roll -o run -- \
          python bench.py --workload $w --mode rollout --steps 600 --warmup 60 $B > $P.fetch_roll.log 2>&1
      run timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/pmc_write_roll -o run -- \
          python bench.py --workload $w --mode rollout --steps 600 --warmup 60 $B > $P.write_roll.log 2>&1
      run timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace_pol -o run -- \
          python bench.py --workload $w --mode policy --steps 600 --warmup 60 $B > $P.trace_pol.log 2>&1
      run timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/pmc_fetch_pol -o run -- \
          python bench.py --workload $w --mode policy --steps 600 --warmup 60 $B > $P.fetch_pol.log 2>&1
      run timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/pmc_write_pol -o run -- \
          python bench.py --workload $w --mode policy --steps 600 --warmup 60 $B > $P.write_pol.log 2>&1
    done ;;
  trace3)
    # two more kernel-trace runs of each step bench (trace_2, trace_3): a
    # dispatch's rocprofv3 mean moves by up to ~8 % between processes on one
    # box (profiles/r06/split_dec/rocprof_ab.md), so collect_round.py keeps the
    # median of the three runs
    for w in $WLS; do
      P=$OUT/prof_$w
      for r in 2 3; do
        run timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace_$r -o run -- \
            python bench.py --workload $w --steps 1000 --warmup 50 $B > $P.trace_$r.log 2>&1
      done
    done ;;
  sq)
    # Newsvendor step (nv_step1_kernel) and rollout (nv_roll_kernel): issue vs wait
    P=$OUT/sq_newsvendor
    for m in step rollout; do
      S="--steps 200 --warmup 20"; [ $m = rollout ] && S="--mode rollout --steps 600 --warmup 60"
      run timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_VMEM \
          --output-format csv -d $P/$m.a -o run -- python bench.py --workload newsvendor $S $B > $P.$m.a.log 2>&1
      run timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT \
          --output-format csv -d $P/$m.b -o run -- python bench.py --workload newsvendor $S $B > $P.$m.b.log 2>&1
    done ;;
  esac
done
echo "gpu_round $TAG done"
