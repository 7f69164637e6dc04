#!/bin/bash
# A/B of the bench's episode fold placement (side stream / inline / none), same box
set -o pipefail
O=gpurun_out/fold_ab
mkdir -p $O
for rep in 1 2; do
for f in inline none; do
  for m in step rollout; do
    timeout -k 10 120 python bench.py --fold $f --mode $m --no-cpu-baseline --no-rollout-line > $O/$m.$f.$rep.json 2>/dev/null || exit 1
  done
  timeout -k 10 120 python bench.py --fold $f --workload invmgmt_lostsales --no-cpu-baseline --no-rollout-line > $O/ls.$f.$rep.json 2>/dev/null || exit 1
done
done
python - <<'PY'
import json,glob
for f in sorted(glob.glob("gpurun_out/fold_ab/*.json")):
    d=json.loads(open(f).read().strip().splitlines()[-1]); r=d["roofline"]
    print(f.split("/")[-1], "%.3f G" % (d["value"]/1e9), "k=%.2fus" % (r["kernel_ms_mean"]*1e3), "fk=%.3f fw=%.3f" % (r["frac_kernel"], r["frac_wall"]))
PY
