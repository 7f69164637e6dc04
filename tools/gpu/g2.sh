#!/bin/bash
# im_roll3o two groups per 6-wave workgroup (INVSIM_IM_ROLL3O_G2) + rollout ablations, LostSales 32768
set -o pipefail
mkdir -p gpurun_out/g2
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -m gpu -k "three_role_rollout_equals_two_role" > gpurun_out/g2/pytest.log 2>&1 || { tail -40 gpurun_out/g2/pytest.log; exit 1; }
tail -2 gpurun_out/g2/pytest.log
L=or-gym-inventory_amd/invsim/_lib/ablate
bash tools/ab.sh invmgmt_lostsales rollout cur INVSIM_IM_ROLL3O_G2=1 $L/libinvsim_ROLL_NO_DRAW.so $L/libinvsim_ROLL_NO_STORE.so | tee gpurun_out/g2/ab.txt
