#!/bin/bash
# Round 4, session c: GPU suite on the 4-role Newsvendor rollout and the staged
# Net 3-role rollout; A/B against the round-start kernels (ablate/NOSTAGE);
# the 4-role timeline.
set -u
OUT=gpurun_out/r04c
mkdir -p $OUT
export TMPDIR=/tmp
run() { echo "+ $*" >&2; "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" >&2; exit $rc; fi; }
run timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
tail -2 $OUT/pytest_gpu.log
OLD=or-gym-inventory_amd/invsim/_lib/ablate/libinvsim_NOSTAGE.so
for w in newsvendor net_backlog; do
  for m in rollout policy; do
    R="--workload $w --mode $m --steps 1200 --warmup 60 --no-cpu-baseline"
    for i in 1 2; do
      run timeout -k 10 120 python bench.py $R > $OUT/${w}_${m}_new.$i.json 2>>$OUT/bench_err.log
      INVSIM_LIB=$OLD run timeout -k 10 120 python bench.py $R > $OUT/${w}_${m}_old.$i.json 2>>$OUT/bench_err.log
    done
  done
done
INVSIM_LIB=or-gym-inventory_amd/invsim/_lib/ablate/libinvsim_TIMING.so run timeout -k 10 120 python tools/timing_nv_roll.py > $OUT/nv_roll_timeline.txt 2>&1
echo r04c done
