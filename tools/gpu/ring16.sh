#!/bin/bash
# the 16-bit action_log ring: the whole GPU suite (with the wide-order oracle test), then A/B against the 32-bit ring build
set -o pipefail
mkdir -p gpurun_out/ring16
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ring16/pytest.log 2>&1 || { tail -40 gpurun_out/ring16/pytest.log; exit 1; }
tail -2 gpurun_out/ring16/pytest.log
if [ -f or-gym-inventory_amd/invsim/_lib/ab/libinvsim_old.so ]; then
  for w in invmgmt_backlog invmgmt_lostsales; do
    bash tools/ab.sh $w step cur or-gym-inventory_amd/invsim/_lib/ab/libinvsim_old.so | tee gpurun_out/ring16/ab_${w}_step.txt
    bash tools/ab.sh $w rollout cur or-gym-inventory_amd/invsim/_lib/ab/libinvsim_old.so | tee gpurun_out/ring16/ab_${w}_rollout.txt
  done
fi
