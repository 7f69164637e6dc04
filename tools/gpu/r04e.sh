#!/bin/bash
# Round 4, session e: the Newsvendor rollout's PTRS role on two lane-pair waves
# (5 waves per workgroup) -- Newsvendor GPU tests, A/B against the 4-wave
# kernel (ablate/NVPAIR0), the 5-wave timeline, then the whole GPU suite.
set -u
OUT=gpurun_out/r04e
mkdir -p $OUT
export TMPDIR=/tmp
run() { echo "+ $*" >&2; "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" >&2; exit $rc; fi; }
run timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "newsvendor or nv_" > $OUT/pytest_nv.log 2>&1
tail -2 $OUT/pytest_nv.log
A=or-gym-inventory_amd/invsim/_lib/ablate
for m in rollout policy; do
  R="--workload newsvendor --mode $m --steps 1200 --warmup 60 --no-cpu-baseline"
  for i in 1 2; do
    run timeout -k 10 120 python bench.py $R > $OUT/nv_${m}_pair.$i.json 2>>$OUT/bench_err.log
    INVSIM_LIB=$A/libinvsim_NVPAIR0.so run timeout -k 10 120 python bench.py $R > $OUT/nv_${m}_four.$i.json 2>>$OUT/bench_err.log
  done
done
INVSIM_LIB=$A/libinvsim_TIMING.so run timeout -k 10 120 python tools/timing_nv_roll.py 5 > $OUT/nv_roll_timeline.txt 2>&1
run timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
tail -2 $OUT/pytest_gpu.log
echo r04e done
