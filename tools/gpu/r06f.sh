#!/bin/bash
# Round 6: the 16-lane-row Net rollout (net_rollq_kernel): parity tests, then
# the K=30 rollout at small shards against the 3-role kernel.
set -u
OUT=gpurun_out/r06f
mkdir -p $OUT
run() { echo "+ $*" >&2; "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" >&2; exit $rc; fi; }
run timeout -k 10 300 python -u -m pytest tests/test_gpu_net_small.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest_small.log 2>&1
tail -3 $OUT/pytest_small.log
B="--workload net_backlog --mode rollout --steps 1200 --warmup 60 --no-cpu-baseline"
for n in 4096 8192 16384; do
  for q in 0 100000; do
    INVSIM_NET_ROLLQ_MAX_N=$q run timeout -k 10 120 python bench.py $B --n-envs $n > $OUT/q${q}_$n.json 2>$OUT/q${q}_$n.err
  done
done
python - <<'PY'
import json
for n in (4096, 8192, 16384):
    row = []
    for q in (0, 100000):
        d = json.loads(open(f"gpurun_out/r06f/q{q}_{n}.json").read().splitlines()[-1])
        row.append(f'{"rollq" if q else "roll3o"} {d["value"]/1e9:.2f}G {d["roofline"]["kernel_ms_mean"]*1e3:.1f}us')
    print(n, " | ".join(row))
PY
