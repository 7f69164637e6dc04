#!/bin/bash
# One GPU session for a round: GPU tests, bench lines for every workload
# (step + rollout), rocprofv3 kernel-trace stats and separate FETCH_SIZE /
# WRITE_SIZE passes per workload.  Everything lands in gpurun_out/round_TAG/.
# Stops at the first failing step (no GPU work after a fault/timeout).
#   tools/gpu_round.sh TAG [tests|bench|prof ...]   (default: all three)
set -u
TAG=${1:-r01}; shift || true
PARTS=${*:-tests bench prof}
OUT=gpurun_out/round_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
run() {
    echo "+ $*" >&2
    "$@"
    rc=$?
    if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" >&2; exit $rc; fi
}
WLS="invmgmt_backlog invmgmt_lostsales newsvendor net_backlog"
for part in $PARTS; do
  case $part in
  tests)
    run timeout -k 10 480 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
    tail -2 $OUT/pytest_gpu.log ;;
  bench)
    run timeout -k 10 180 python bench.py > $OUT/bench_default.log 2>&1
    tail -1 $OUT/bench_default.log
    for w in $WLS; do
      run timeout -k 10 120 python bench.py --workload $w --no-cpu-baseline > $OUT/bench_${w}_step.log 2>&1
      run timeout -k 10 120 python bench.py --workload $w --mode rollout --steps 1200 --no-cpu-baseline \
          > $OUT/bench_${w}_rollout.log 2>&1
      tail -n1 $OUT/bench_${w}_step.log | cut -c1-200
    done ;;
  prof)
    for w in $WLS; do
      P=$OUT/prof_$w
      run timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace -o run -- \
          python bench.py --workload $w --steps 1000 --warmup 50 --no-cpu-baseline > $P.trace.log 2>&1
      run timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace_roll -o run -- \
          python bench.py --workload $w --mode rollout --steps 600 --warmup 60 --no-cpu-baseline > $P.trace_roll.log 2>&1
      run timeout -k 10 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/pmc_fetch -o run -- \
          python bench.py --workload $w --steps 200 --warmup 20 --no-cpu-baseline > $P.fetch.log 2>&1
      run timeout -k 10 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/pmc_write -o run -- \
          python bench.py --workload $w --steps 200 --warmup 20 --no-cpu-baseline > $P.write.log 2>&1
    done ;;
  esac
done
echo "gpu_round $TAG done"
