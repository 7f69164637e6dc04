#!/bin/bash
# A/B benchmark of library builds in one GPU session (alternating runs).
#   tools/ab.sh WORKLOAD MODE LIB... (paths; "cur" = the in-tree build)
set -u
W=$1; M=$2; shift 2
for rep in 1 2 3; do
  for L in "$@"; do
    [ "$L" = cur ] && P=or-gym-inventory_amd/invsim/_lib/libinvsim.so || P=$L
    INVSIM_LIB=$P timeout -k 10 100 python bench.py --workload $W --mode $M --steps 1500 --no-cpu-baseline \
        > gpurun_out/ab.log 2>&1 || exit 1
    echo "$rep $(basename $P) $(tail -1 gpurun_out/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e9,3), round(d["roofline"]["kernel_ms_mean"]*1e3,2))')"
  done
done
