#!/bin/bash
# 3-role rollout kernels above their default batch thresholds (65536 envs)
set -u
OUT=gpurun_out/thr; mkdir -p $OUT
b() { timeout -k 10 100 python bench.py --workload $1 --mode rollout --steps 1200 --no-cpu-baseline --n-envs 65536 > $OUT/r.log 2>&1 || { tail $OUT/r.log; exit 1; }
      echo "$1 $2 $(tail -1 $OUT/r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e9,3), round(d["roofline"]["kernel_ms_mean"]*1e3,2))')"; }
for rep in 1 2; do
  b invmgmt_backlog default
  INVSIM_IM_ROLL3O_MAX_N=65536 b invmgmt_backlog roll3o
  b net_backlog default
  INVSIM_NET_ROLL3=1 b net_backlog roll3o
done
