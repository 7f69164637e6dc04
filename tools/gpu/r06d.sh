#!/bin/bash
# Round 6: end-of-region wait (hipEventSynchronize vs hipEventQuery polling vs
# device synchronize) on the driver-style line, three runs each, interleaved.
set -u
OUT=gpurun_out/r06d
mkdir -p $OUT
run() { echo "+ $*" >&2; "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" >&2; exit $rc; fi; }
B="--no-cpu-baseline --no-config-lines --no-graph-line"
for i in 1 2 3; do
  for st in event spin sync; do
    run timeout -k 10 120 python bench.py --steps 20 --warmup 5 --stop $st $B > $OUT/${st}_$i.json 2>$OUT/${st}_$i.err
  done
done
python - <<'PY'
import json
for st in ("event", "spin", "sync"):
    row = []
    for i in (1, 2, 3):
        d = json.loads(open(f"gpurun_out/r06d/{st}_{i}.json").read().splitlines()[-1])
        row.append(f'{d["value"]/1e9:.3f}G {d["ms_per_step"]*1e3:.3f}/{d["roofline"]["kernel_ms_mean"]*1e3:.3f}us roll {d["rollout"]["value"]/1e9:.2f}G {d["rollout"]["episode_stats"]["fold"]}')
    print(st, " | ".join(row))
PY
