#!/bin/bash
# im_roll3o with the actions staged through the demand wave: rollout tests, then A/B
set -o pipefail
O=gpurun_out/stage
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_policies.py tests/test_gpu_fast_stream.py -x -v --timeout 200 --timeout-method thread -m gpu -k "rollout or three_role or policy or fused or flat" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash tools/ab.sh invmgmt_lostsales rollout cur INVSIM_IM_ROLL3O_G2=1 | tee $O/ab_ls.txt
bash tools/ab.sh invmgmt_lostsales policy cur INVSIM_IM_ROLL3O_G2=1 | tee $O/ab_ls_pol.txt
