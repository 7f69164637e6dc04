#!/bin/bash
# Round 4, session d: GPU suite on the reverted Net rollout; s_setprio A/B of
# the Newsvendor stream waves (ablate/PRIO); per-role barrier-wait timelines
# of the NV 4-role and IM 3-role rollouts (ablate/TIMING).
set -u
OUT=gpurun_out/r04d
mkdir -p $OUT
export TMPDIR=/tmp
run() { echo "+ $*" >&2; "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" >&2; exit $rc; fi; }
run timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
tail -2 $OUT/pytest_gpu.log
A=or-gym-inventory_amd/invsim/_lib/ablate
T=$A/libinvsim_TIMING.so
INVSIM_LIB=$T run timeout -k 10 120 python tools/timing_nv_roll.py > $OUT/nv_roll_timeline.txt 2>&1
INVSIM_LIB=$T run timeout -k 10 120 python tools/timing_im_roll.py 32768 > $OUT/im_roll_timeline.txt 2>&1
INVSIM_LIB=$T run timeout -k 10 120 python tools/timing_im_roll.py 32768 policy > $OUT/im_roll_policy_timeline.txt 2>&1
for m in rollout policy; do
  R="--workload newsvendor --mode $m --steps 1200 --warmup 60 --no-cpu-baseline"
  for i in 1 2; do
    run timeout -k 10 120 python bench.py $R > $OUT/nv_${m}_base.$i.json 2>>$OUT/bench_err.log
    INVSIM_LIB=$A/libinvsim_PRIO.so run timeout -k 10 120 python bench.py $R > $OUT/nv_${m}_prio.$i.json 2>>$OUT/bench_err.log
  done
done
echo r04d done
