set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -m gpu -k "rollout or register_window or lookahead or policy" > gpurun_out/t_roll.log 2>&1 || { tail -40 gpurun_out/t_roll.log; exit 1; }
tail -3 gpurun_out/t_roll.log
timeout -k 10 300 python -u -m pytest tests/test_policies.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/t_roll2.log 2>&1 || { tail -40 gpurun_out/t_roll2.log; exit 1; }
tail -2 gpurun_out/t_roll2.log
bash tools/ab.sh invmgmt_backlog rollout cur INVSIM_IM_ROLL=0
bash tools/ab.sh invmgmt_lostsales rollout cur INVSIM_IM_ROLL=0
