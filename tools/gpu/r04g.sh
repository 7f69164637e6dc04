#!/bin/bash
# Round 4, session g: the Newsvendor rollout's PTRS wave through ptrs_decide
# (branch-light candidate) -- Newsvendor GPU tests, A/B against the branchy
# body (ablate/PTRSOLD).
set -u
OUT=gpurun_out/r04g
mkdir -p $OUT
export TMPDIR=/tmp
run() { echo "+ $*" >&2; "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" >&2; exit $rc; fi; }
run timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "newsvendor or nv_" > $OUT/pytest_nv.log 2>&1
tail -2 $OUT/pytest_nv.log
A=or-gym-inventory_amd/invsim/_lib/ablate
for m in rollout policy; do
  R="--workload newsvendor --mode $m --steps 1200 --warmup 60 --no-cpu-baseline"
  for i in 1 2; do
    run timeout -k 10 120 python bench.py $R > $OUT/nv_${m}_decide.$i.json 2>>$OUT/bench_err.log
    INVSIM_LIB=$A/libinvsim_PTRSOLD.so run timeout -k 10 120 python bench.py $R > $OUT/nv_${m}_old.$i.json 2>>$OUT/bench_err.log
  done
done
echo r04g done
