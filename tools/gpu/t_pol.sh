set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_policies.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -m gpu -k "constant or policy or net" > gpurun_out/t_pol.log 2>&1 || { tail -60 gpurun_out/t_pol.log; exit 1; }
tail -5 gpurun_out/t_pol.log
