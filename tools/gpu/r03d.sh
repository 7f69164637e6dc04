#!/bin/bash
# round 3 session d: the whole GPU suite, then the round's bench / profile / SQ passes
set -o pipefail
O=gpurun_out/r03d
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
bash tools/gpu_round.sh r03d bench prof sq || exit 1
timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || exit 1
cut -c1-300 $O/bench_driver.json
