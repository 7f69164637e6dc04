set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_newsvendor_info.py tests/test_gpu_bench.py tests/test_compat.py -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/t_new.log 2>&1 || { tail -60 gpurun_out/t_new.log; exit 1; }
tail -15 gpurun_out/t_new.log
