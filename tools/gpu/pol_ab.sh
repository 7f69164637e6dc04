#!/bin/bash
# in-kernel policy on the fused rollout kernel vs the run kernel
set -o pipefail
O=gpurun_out/pol_ab
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_policies.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for w in newsvendor invmgmt_backlog invmgmt_lostsales net_backlog; do
  for r in 1 0; do
    INVSIM_IM_POL_ROLL=$r INVSIM_NET_POL_ROLL=$r INVSIM_NV_POL_ROLL=$r timeout -k 10 120 python bench.py --workload $w --mode policy --no-cpu-baseline --no-rollout-line > $O/$w.$r.json 2>/dev/null || exit 1
  done
done
python - <<'PY'
import json,glob
for f in sorted(glob.glob("gpurun_out/pol_ab/*.json")):
    d=json.loads(open(f).read().strip().splitlines()[-1]); r=d["roofline"]
    print(f.split("/")[-1], "%.3f G" % (d["value"]/1e9), "k=%.2fus" % (r["kernel_ms_mean"]*1e3), "fk=%.3f fw=%.3f" % (r["frac_kernel"], r["frac_wall"]))
PY
