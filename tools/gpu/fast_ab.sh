#!/bin/bash
# fast (Philox) stream on the fused kernels: tests, then numpy vs philox bench lines
set -o pipefail
O=gpurun_out/fast_ab
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_fast_stream.py -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for w in ${WLS:-invmgmt_backlog invmgmt_lostsales net_backlog}; do
  for ds in numpy philox; do
    for m in step policy; do
      timeout -k 10 120 python bench.py --workload $w --demand-stream $ds --mode $m --no-cpu-baseline > $O/${w}_${ds}_${m}.json 2> $O/${w}_${ds}_${m}.err || { tail -20 $O/${w}_${ds}_${m}.err; exit 1; }
    done
  done
done
python - <<'PY'
import json,glob
for f in sorted(glob.glob("gpurun_out/fast_ab/*.json")):
    d=json.loads(open(f).read().strip().splitlines()[-1]); r=d["roofline"]; ro=d.get("rollout") or {}
    s = f.split("/")[-1] + " %.2f G k=%.2fus fk=%.3f" % (d["value"]/1e9, r["kernel_ms_mean"]*1e3, r["frac_kernel"])
    if ro: s += " | roll %.2f G %.1fus" % (ro["value"]/1e9, ro["roofline"]["kernel_ms_mean"]*1e3)
    print(s)
PY
