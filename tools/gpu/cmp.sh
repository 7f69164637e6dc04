set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_policies.py -x -q --timeout 300 --timeout-method thread -m gpu -k "net" > gpurun_out/t_cmp.log 2>&1 || { tail -40 gpurun_out/t_cmp.log; exit 1; }
tail -2 gpurun_out/t_cmp.log
A=or-gym-inventory_amd/invsim/_lib/ablate
bash tools/ab.sh net_backlog step cur $A/libinvsim_OLD.so
