#!/bin/bash
# two-group 3-role kernel as the policy-rollout default: policy tests, then A/B
set -o pipefail
mkdir -p gpurun_out/g2pol
timeout -k 10 400 python -u -m pytest tests/test_policies.py tests/test_gpu_parity.py tests/test_gpu_graphs.py tests/test_gpu_distributed.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/g2pol/pytest.log 2>&1 || { tail -40 gpurun_out/g2pol/pytest.log; exit 1; }
tail -2 gpurun_out/g2pol/pytest.log
bash tools/ab.sh invmgmt_lostsales policy cur INVSIM_IM_ROLL3O_G2=0 | tee gpurun_out/g2pol/ab_lostsales_policy.txt
bash tools/ab.sh invmgmt_lostsales rollout cur INVSIM_IM_ROLL3O_G2=1 | tee gpurun_out/g2pol/ab_lostsales_rollout.txt
