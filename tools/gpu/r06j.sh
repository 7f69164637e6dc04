#!/bin/bash
# Round 6: net_roll4_kernel (profit on its own wave): parity, then the K=30
# rollout at 4 096 - 16 384 envs against net_roll3o_kernel.
set -u
OUT=gpurun_out/r06j
mkdir -p $OUT
run() { echo "+ $*" >&2; "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" >&2; exit $rc; fi; }
run timeout -k 10 400 python -u -m pytest tests/test_gpu_net_small.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest_small.log 2>&1
tail -2 $OUT/pytest_small.log
B="--workload net_backlog --mode rollout --steps 1200 --warmup 60 --no-cpu-baseline"
for i in 1 2; do
for n in 4096 8192 16384; do
  for q in 0 100000; do
    INVSIM_NET_ROLL4_MAX_N=$q run timeout -k 10 120 python bench.py $B --n-envs $n > $OUT/q${q}_${n}_$i.json 2>$OUT/q${q}_${n}_$i.err
  done
done
done
python - <<'PY'
import json
for n in (4096, 8192, 16384):
    row = []
    for q in (0, 100000):
        for i in (1, 2):
            d = json.loads(open(f"gpurun_out/r06j/q{q}_{n}_{i}.json").read().splitlines()[-1])
            row.append(f'{"roll4" if q else "roll3o"} {d["value"]/1e9:.2f}G {d["roofline"]["kernel_ms_mean"]*1e3:.1f}us')
    print(n, " | ".join(row))
PY
