set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 python -u -m pytest tests/test_gpu_vector.py tests/test_gpu_bench.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/t_rx.log 2>&1 || { tail -30 gpurun_out/t_rx.log; exit 1; }
tail -1 gpurun_out/t_rx.log
timeout -k 10 200 python tools/py_overhead.py > gpurun_out/pyo.log 2>&1 || exit 1
cat gpurun_out/pyo.log
timeout -k 10 120 rocprofv3 --marker-trace --kernel-trace --stats --output-format csv -d gpurun_out/mk -o run -- python bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/mk.log 2>&1 || exit 1
ls gpurun_out/mk
