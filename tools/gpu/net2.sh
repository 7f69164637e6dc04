#!/bin/bash
# Net rollout tests, then the 2-role kernel at 65536 envs (INVSIM_NET_ROLL3=0) against $1.
set -u
OUT=gpurun_out/net2; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "net" > $OUT/pytest_net.log 2>&1 || { tail -30 $OUT/pytest_net.log; exit 1; }
tail -1 $OUT/pytest_net.log
for rep in 1 2; do for L in or-gym-inventory_amd/invsim/_lib/libinvsim.so $1; do
  INVSIM_LIB=$L timeout -k 10 100 python bench.py --workload net_backlog --n-envs 65536 --mode rollout --steps 1200 --no-cpu-baseline > $OUT/r.log 2>&1 || { tail $OUT/r.log; exit 1; }
  echo "$L $(tail -1 $OUT/r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e9,3), round(d["roofline"]["kernel_ms_mean"]*1e3,2))')"
done; done
