#!/bin/bash
# round 3 final session, part 1: the whole GPU suite, bench lines, the driver-style line
set -o pipefail
O=gpurun_out/round_r03h
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
bash tools/gpu_round.sh r03h bench || exit 1
timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || exit 1
cut -c1-300 $O/bench_driver.json
