set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -m gpu -k "newsvendor" > gpurun_out/t_nv.log 2>&1 || { tail -40 gpurun_out/t_nv.log; exit 1; }
tail -3 gpurun_out/t_nv.log
A=or-gym-inventory_amd/invsim/_lib/ablate
bash tools/ab.sh newsvendor rollout cur $A/libinvsim_NVCH16.so $A/libinvsim_ROLL_NO_MULT.so
