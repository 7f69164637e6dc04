#!/bin/bash
# the fused policy test with the two-group 3-role leg; A/B of the split step without its window read (ablation)
set -o pipefail
mkdir -p gpurun_out/nw
timeout -k 10 300 python -u -m pytest tests/test_policies.py -x -q --timeout 200 --timeout-method thread -m gpu -k "fused" > gpurun_out/nw/pytest.log 2>&1 || { tail -40 gpurun_out/nw/pytest.log; exit 1; }
tail -2 gpurun_out/nw/pytest.log
for w in invmgmt_backlog invmgmt_lostsales; do
  bash tools/ab.sh $w step cur or-gym-inventory_amd/invsim/_lib/ab/libinvsim_NW.so | tee gpurun_out/nw/ab_$w.txt
done
