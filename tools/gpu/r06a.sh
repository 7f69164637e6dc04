#!/bin/bash
# Round 6, first session: GPU tests, the driver-style line and the default line.
set -u
OUT=gpurun_out/r06a
mkdir -p $OUT
export TMPDIR=/tmp
run() { echo "+ $*" >&2; "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" >&2; exit $rc; fi; }
run timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
tail -2 $OUT/pytest_gpu.log
run timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/driver_style.json 2>$OUT/driver_style.err
run timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/default.json 2>$OUT/default.err
python - <<'PY'
import json
for f in ("driver_style", "default"):
    d = json.loads(open(f"gpurun_out/r06a/{f}.json").read().splitlines()[-1])
    print(f, round(d["value"] / 1e9, 3), "G", round(d["ms_per_step"] * 1e3, 3), "us", d["roofline"]["frac"], d["roofline"].get("hbm_counter", {}).get("frac"))
    for k, v in d.get("configs", {}).items():
        if k != "note":
            print("  ", k, round(v["step"]["value"] / 1e9, 3), round(v["rollout"]["value"] / 1e9, 3), v["step"].get("frac"), v["step"].get("hbm_counter"))
PY
