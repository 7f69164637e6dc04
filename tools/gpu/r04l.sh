#!/bin/bash
# Round 4, session l: the bench's graph region with several cycles per replay
# (one fold per replay) -- the bench GPU tests and the default line twice.
set -u
OUT=gpurun_out/r04l
mkdir -p $OUT
export TMPDIR=/tmp
run() { echo "+ $*" >&2; "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" >&2; exit $rc; fi; }
run timeout -k 10 400 python -u -m pytest tests/test_gpu_bench.py tests/test_gpu_rccl.py tests/test_gpu_graphs.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_bench.log 2>&1
tail -2 $OUT/pytest_bench.log
for i in 1 2; do
  run timeout -k 10 180 python bench.py --no-cpu-baseline > $OUT/bench_default.$i.json 2>>$OUT/bench_err.log
done
echo r04l done
