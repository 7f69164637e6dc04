#!/bin/bash
# Round 4, session j: the Newsvendor PTRS wave software-pipelined (the next
# candidate's uniforms drawn while the pending one is tested) -- Newsvendor
# GPU tests, A/B against one candidate per trip (ablate/NOPIPE), timeline.
set -u
OUT=gpurun_out/r04j
mkdir -p $OUT
export TMPDIR=/tmp
run() { echo "+ $*" >&2; "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" >&2; exit $rc; fi; }
run timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "newsvendor or nv_" > $OUT/pytest_nv.log 2>&1
tail -2 $OUT/pytest_nv.log
A=or-gym-inventory_amd/invsim/_lib/ablate
for m in rollout policy; do
  R="--workload newsvendor --mode $m --steps 1200 --warmup 60 --no-cpu-baseline"
  for i in 1 2; do
    run timeout -k 10 120 python bench.py $R > $OUT/nv_${m}_pipe.$i.json 2>>$OUT/bench_err.log
    INVSIM_LIB=$A/libinvsim_NOPIPE.so run timeout -k 10 120 python bench.py $R > $OUT/nv_${m}_nopipe.$i.json 2>>$OUT/bench_err.log
  done
done
INVSIM_LIB=$A/libinvsim_TIMING.so run timeout -k 10 120 python tools/timing_nv_roll.py L0 > $OUT/nv_roll_timeline.txt 2>&1
echo r04j done
