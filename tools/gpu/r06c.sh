#!/bin/bash
# Round 6: why the eager step region is slower with the episode sink at 2000
# steps: kernel-trace both folds, and the event rate at several region lengths.
set -u
OUT=gpurun_out/r06c
mkdir -p $OUT
export TMPDIR=/tmp
run() { echo "+ $*" >&2; "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" >&2; exit $rc; fi; }
B="--no-cpu-baseline --no-config-lines --no-rollout-line --no-graph-line"
for f in sink inline; do
  for s in 20 200 2000; do
    run timeout -k 10 120 python bench.py --steps $s --warmup 5 --fold $f $B > $OUT/s${s}_$f.json 2>$OUT/s${s}_$f.err
  done
  run timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_$f -o run -- \
      python bench.py --steps 1000 --warmup 50 --fold $f $B > $OUT/trace_$f.log 2>&1
done
python - <<'PY'
import json, glob, csv
for f in ("sink", "inline"):
    for s in (20, 200, 2000):
        d = json.loads(open(f"gpurun_out/r06c/s{s}_{f}.json").read().splitlines()[-1])
        print(f, s, round(d["ms_per_step"] * 1e3, 3), round(d["roofline"]["kernel_ms_mean"] * 1e3, 3))
    for p in glob.glob(f"gpurun_out/r06c/trace_{f}/**/*kernel_stats.csv", recursive=True):
        for r in csv.DictReader(open(p)):
            print("   ", r["Name"][:90], r["Calls"], r["AverageNs"])
PY
