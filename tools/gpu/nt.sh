#!/bin/bash
# A/B: non-temporal state stores (make nt) and lookahead workgroups last, InvMgmt steps
set -o pipefail
mkdir -p gpurun_out/nt
for w in invmgmt_backlog invmgmt_lostsales; do
  bash tools/ab.sh $w step cur or-gym-inventory_amd/invsim/_lib/ab/libinvsim_NT.so INVSIM_IM_LA_LAST=1 | tee gpurun_out/nt/ab_$w.txt
done
