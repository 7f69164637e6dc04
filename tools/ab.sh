#!/bin/bash
# A/B benchmark of library builds / env settings in one GPU session (alternating runs).
#   tools/ab.sh WORKLOAD MODE ARM...
# ARM: a library path, "cur" (the in-tree build), or VAR=VALUE (in-tree build
# with that environment variable set)
set -u
W=$1; M=$2; shift 2
for rep in 1 2 3; do
  for A in "$@"; do
    P=or-gym-inventory_amd/invsim/_lib/libinvsim.so; E=INVSIM_AB_NONE=1
    case "$A" in
      cur) ;;
      *=*) E=$A ;;
      *) P=$A ;;
    esac
    env "$E" INVSIM_LIB=$P timeout -k 10 100 python bench.py --workload $W --mode $M --steps 1500 --no-cpu-baseline \
        > gpurun_out/ab.log 2>&1 || exit 1
    echo "$rep $A $(tail -1 gpurun_out/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e9,3), round(d["roofline"]["kernel_ms_mean"]*1e3,2))')"
  done
done
