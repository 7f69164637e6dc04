#!/bin/bash
# A/B of library builds at a given batch size (alternating runs, 3 reps).
#   tools/ab_n.sh WORKLOAD MODE N ARM...     ARM: a library path, "cur", or
#   "VAR=VALUE" (the current library with that INVSIM_* switch set)
set -u
W=$1; M=$2; N=$3; shift 3
for rep in 1 2 3; do
  for A in "$@"; do
    P=or-gym-inventory_amd/invsim/_lib/libinvsim.so
    E=INVSIM_AB_ARM=1
    case $A in cur) ;; *=*) E=$A ;; *) P=$A ;; esac
    env INVSIM_LIB=$P $E timeout -k 10 120 python bench.py --workload $W --mode $M --n-envs $N --steps 1200 \
        --no-cpu-baseline --no-rollout-line --no-graph-line > gpurun_out/ab_n.log 2>&1 || exit 1
    echo "$rep $(basename $A) $(tail -1 gpurun_out/ab_n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e9,3), round(d["roofline"]["kernel_ms_mean"]*1e3,2))')"
  done
done
