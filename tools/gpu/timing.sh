#!/bin/bash
# per-wave timeline of the InvMgmt split step (TIMING build) at 65 536 and 32 768 envs
set -o pipefail
mkdir -p gpurun_out/timing
for n in 65536 32768; do
  INVSIM_LIB=or-gym-inventory_amd/invsim/_lib/ab/libinvsim_TIMING.so timeout -k 10 120 python tools/timing_im_step.py $n > gpurun_out/timing/im_step_$n.txt 2>&1 || { cat gpurun_out/timing/im_step_$n.txt; exit 1; }
  cat gpurun_out/timing/im_step_$n.txt
done
