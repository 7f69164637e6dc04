#!/bin/bash
# Round 4, session a: full GPU suite (new parity / RCCL / fast-stream / bench
# tests), driver-style bench lines with both region stops, the closing-wait
# variants, and the per-launch floor eager vs graph replay.
set -u
OUT=gpurun_out/r04a
mkdir -p $OUT
export TMPDIR=/tmp
run() { echo "+ $*" >&2; "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" >&2; exit $rc; fi; }
run timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
tail -2 $OUT/pytest_gpu.log
for i in 1 2; do
  run timeout -k 10 120 python bench.py --steps 20 --warmup 5 --stop event > $OUT/bench_driver_event.$i.json 2>$OUT/bench_err.log
  run timeout -k 10 120 python bench.py --steps 20 --warmup 5 --stop sync --no-cpu-baseline > $OUT/bench_driver_sync.$i.json 2>>$OUT/bench_err.log
done
run timeout -k 10 120 python tools/sync_overhead.py > $OUT/sync_overhead.txt 2>&1
run timeout -k 10 60 tools/dispatch_cost graph > $OUT/dispatch_cost_graph.txt 2>&1
run timeout -k 10 180 python tools/graph_floor.py > $OUT/graph_floor.txt 2>&1
echo r04a done
