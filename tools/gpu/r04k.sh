#!/bin/bash
# Round 4, session k: the InvMgmt split step with 32 envs per workgroup for
# batches <= 32768 -- InvMgmt GPU tests, A/B against 64 (INVSIM_IM_EG=64) on
# the LostSales 32768 step, and the 65536-env Backlog step unchanged.
set -u
OUT=gpurun_out/r04k
mkdir -p $OUT
export TMPDIR=/tmp
run() { echo "+ $*" >&2; "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" >&2; exit $rc; fi; }
run timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "invmgmt or im_ or split or lookahead" > $OUT/pytest_im.log 2>&1
tail -2 $OUT/pytest_im.log
S="--workload invmgmt_lostsales --no-cpu-baseline --no-rollout-line --no-graph-line"
for i in 1 2; do
  run timeout -k 10 120 python bench.py $S > $OUT/ls_step_eg32.$i.json 2>>$OUT/bench_err.log
  INVSIM_IM_EG=64 run timeout -k 10 120 python bench.py $S > $OUT/ls_step_eg64.$i.json 2>>$OUT/bench_err.log
done
B="--workload invmgmt_backlog --no-cpu-baseline --no-rollout-line --no-graph-line"
for i in 1 2; do
  run timeout -k 10 120 python bench.py $B > $OUT/bl_step_eg64.$i.json 2>>$OUT/bench_err.log
  INVSIM_IM_EG=32 run timeout -k 10 120 python bench.py $B > $OUT/bl_step_eg32.$i.json 2>>$OUT/bench_err.log
done
echo r04k done
