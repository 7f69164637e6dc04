#!/bin/bash
# Round 6: the episode sink -- its GPU tests, the episode-fold tests, then the
# driver-style line with the fold (side-by-side) and with the fused sink.
set -u
OUT=gpurun_out/r06b
mkdir -p $OUT
export TMPDIR=/tmp
run() { echo "+ $*" >&2; "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" >&2; exit $rc; fi; }
run timeout -k 10 300 python -u -m pytest tests/test_gpu_episode_sink.py tests/test_gpu_episode_fold.py tests/test_gpu_rccl.py tests/test_gpu_long_draws.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest_sink.log 2>&1
tail -3 $OUT/pytest_sink.log
for f in inline sink; do
  run timeout -k 10 300 python bench.py --steps 20 --warmup 5 --fold $f --no-cpu-baseline --no-config-lines > $OUT/driver_$f.json 2>$OUT/driver_$f.err
  run timeout -k 10 300 python bench.py --fold $f --no-cpu-baseline --no-config-lines > $OUT/default_$f.json 2>$OUT/default_$f.err
done
python - <<'PY'
import json
for f in ("driver_inline", "driver_sink", "default_inline", "default_sink"):
    d = json.loads(open(f"gpurun_out/r06b/{f}.json").read().splitlines()[-1])
    r = d["rollout"]
    print(f, round(d["value"] / 1e9, 3), "G", round(d["ms_per_step"] * 1e3, 3), "us wall", round(d["roofline"]["kernel_ms_mean"] * 1e3, 3), "us ev",
          "| rollout", round(r["value"] / 1e9, 3), round(r["roofline"]["kernel_ms_mean"] * 1e3, 2), "| ep", d["episode_stats"]["episodes"], r["episode_stats"]["episodes"], r["episode_stats"]["mean_return"])
PY
