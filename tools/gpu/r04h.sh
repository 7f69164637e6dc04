#!/bin/bash
# Round 4, session h: every PTRS candidate through ptrs_decide (IM / Net flat
# loops, the compacted lookaheads, the Newsvendor waves) -- the whole GPU
# suite, then A/B against the branchy body (ablate/PTRSOLD) on each workload.
set -u
OUT=gpurun_out/r04h
mkdir -p $OUT
export TMPDIR=/tmp
run() { echo "+ $*" >&2; "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" >&2; exit $rc; fi; }
run timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
tail -2 $OUT/pytest_gpu.log
OLD=or-gym-inventory_amd/invsim/_lib/ablate/libinvsim_PTRSOLD.so
for w in invmgmt_backlog invmgmt_lostsales newsvendor net_backlog; do
  S="--workload $w --no-cpu-baseline --no-rollout-line --no-graph-line"
  R="--workload $w --mode rollout --steps 1200 --warmup 60 --no-cpu-baseline"
  for i in 1 2; do
    run timeout -k 10 120 python bench.py $S > $OUT/${w}_step_new.$i.json 2>>$OUT/bench_err.log
    INVSIM_LIB=$OLD run timeout -k 10 120 python bench.py $S > $OUT/${w}_step_old.$i.json 2>>$OUT/bench_err.log
    run timeout -k 10 120 python bench.py $R > $OUT/${w}_roll_new.$i.json 2>>$OUT/bench_err.log
    INVSIM_LIB=$OLD run timeout -k 10 120 python bench.py $R > $OUT/${w}_roll_old.$i.json 2>>$OUT/bench_err.log
  done
done
echo r04h done
