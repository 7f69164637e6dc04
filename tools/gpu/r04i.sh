#!/bin/bash
# Round 4, session i: Newsvendor rollout layout 1 (two PTRS lane-pair waves,
# the multiplication draws in the obs wave) -- Newsvendor GPU tests, A/B
# against layout 0 (ablate/NVL0), the layout-1 timeline.
set -u
OUT=gpurun_out/r04i
mkdir -p $OUT
export TMPDIR=/tmp
run() { echo "+ $*" >&2; "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" >&2; exit $rc; fi; }
run timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "newsvendor or nv_" > $OUT/pytest_nv.log 2>&1
tail -2 $OUT/pytest_nv.log
A=or-gym-inventory_amd/invsim/_lib/ablate
for m in rollout policy; do
  R="--workload newsvendor --mode $m --steps 1200 --warmup 60 --no-cpu-baseline"
  for i in 1 2; do
    run timeout -k 10 120 python bench.py $R > $OUT/nv_${m}_l1.$i.json 2>>$OUT/bench_err.log
    INVSIM_LIB=$A/libinvsim_NVL0.so run timeout -k 10 120 python bench.py $R > $OUT/nv_${m}_l0.$i.json 2>>$OUT/bench_err.log
  done
done
INVSIM_LIB=$A/libinvsim_TIMING.so run timeout -k 10 120 python tools/timing_nv_roll.py L1 > $OUT/nv_roll_timeline.txt 2>&1
echo r04i done
