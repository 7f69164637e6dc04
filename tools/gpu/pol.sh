set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_policies.py tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -m gpu -k "policies or newsvendor or rollout" > gpurun_out/t_pol.log 2>&1 || { tail -40 gpurun_out/t_pol.log; exit 1; }
tail -3 gpurun_out/t_pol.log
