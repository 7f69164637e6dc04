set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "lookahead or split or rollout_equals or same_step or checkpoint or integers_buffer or many_draws or newsvendor" > gpurun_out/t_la.log 2>&1 || { tail -30 gpurun_out/t_la.log; exit 1; }
tail -3 gpurun_out/t_la.log
bash tools/ab.sh newsvendor step cur INVSIM_NV_AHEAD=0
bash tools/ab.sh invmgmt_backlog step cur
