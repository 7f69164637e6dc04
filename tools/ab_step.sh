#!/bin/bash
# A/B step-mode benches: /tmp/abstep.sh OUT TOGGLE workloads...
OUT=$1; TOGGLE=$2; shift 2
mkdir -p $OUT
for w in $*; do for v in base ab; do
  if [ $v = ab ]; then E="env $TOGGLE"; else E=""; fi
  $E timeout -k 10 120 python bench.py --workload $w --no-cpu-baseline > $OUT/${w}_$v.log 2>&1 || { echo FAILED $w $v; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/${w}_$v.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$w $v', round(d['value']/1e9,3), 'G', round(r['kernel_ms_mean']*1e3,2), 'us', round(r['frac'],3))"
done; done
