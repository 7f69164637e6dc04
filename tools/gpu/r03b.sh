#!/bin/bash
# round 3 session b: fast-stream tests first, then the whole GPU suite, then
# parity vs fast-stream bench lines for InvMgmt and Newsvendor
set -o pipefail
O=gpurun_out/r03b
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_fast_stream.py tests/test_gpu_episode_fold.py -x -v --timeout 120 --timeout-method thread > $O/pytest_fast.log 2>&1 || { tail -40 $O/pytest_fast.log; exit 1; }
tail -2 $O/pytest_fast.log
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
for w in invmgmt_backlog newsvendor invmgmt_lostsales net_backlog; do
  for ds in numpy philox; do
    timeout -k 10 120 python bench.py --workload $w --demand-stream $ds --no-cpu-baseline > $O/bench_${w}_${ds}.json 2> $O/bench_${w}_${ds}.err || { tail -20 $O/bench_${w}_${ds}.err; exit 1; }
  done
done
timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || exit 1
python - <<'PY'
import json,glob
for f in sorted(glob.glob("gpurun_out/r03b/bench_*.json")):
    d=json.load(open(f)); r=d["roofline"]; ro=d.get("rollout",{})
    print(f.split("/")[-1], "%.2f G" % (d["value"]/1e9), "k=%.2fus" % (r["kernel_ms_mean"]*1e3), "fk=%.3f fw=%.3f" % (r["frac_kernel"], r["frac_wall"]),
          "roll %.2f G %.1fus fk=%.3f" % (ro.get("value",0)/1e9, ro.get("roofline",{}).get("kernel_ms_mean",0)*1e3, ro.get("roofline",{}).get("frac_kernel",0)))
PY
