#!/bin/bash
# Net rollout: 3-role kernel parity tests, then A/B against the 2-role kernel.
set -u
OUT=gpurun_out/net3; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "net" > $OUT/pytest_net.log 2>&1 || { tail -30 $OUT/pytest_net.log; exit 1; }
tail -2 $OUT/pytest_net.log
for v in 1 0 1 0; do
  INVSIM_NET_ROLL3=$v timeout -k 10 120 python bench.py --workload net_backlog --mode rollout --steps 1200 --no-cpu-baseline > $OUT/roll_$v.log 2>&1 || exit 1
  echo "ROLL3=$v $(python -c "import json,sys;d=json.loads(open('$OUT/roll_$v.log').read().strip().splitlines()[-1]);print(round(d['value']/1e9,3),'G',round(d['roofline']['kernel_ms_mean']*1e3,2),'us',round(d['roofline']['frac'],3))")"
done
