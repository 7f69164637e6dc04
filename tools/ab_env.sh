#!/bin/bash
# A/B of an environment toggle on rollout benches: tools/ab_env.sh OUTDIR "VAR=1" [workloads...]
# Each bench runs under its own time limit; stops at the first failure.
set -u
OUT=$1; TOGGLE=$2; shift 2
WLS=${*:-invmgmt_backlog invmgmt_lostsales newsvendor net_backlog}
mkdir -p $OUT
for w in $WLS; do
  for v in base ab; do
    if [ $v = ab ]; then E="env $TOGGLE"; else E=""; fi
    $E timeout -k 10 120 python bench.py --workload $w --mode rollout --steps 1200 --no-cpu-baseline > $OUT/${w}_$v.log 2>&1 || { echo "FAILED $w $v"; exit 1; }
    python -c "import json,sys; d=json.loads(open('$OUT/${w}_$v.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$w $v', round(d['value']/1e9,2), 'G', round(r['kernel_ms_mean']*1e3,1), 'us', round(r['frac'],3))"
  done
done
