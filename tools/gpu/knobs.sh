#!/bin/bash
# per-launch overhead of back-to-back dependent launches under HIP runtime knobs
set -o pipefail
O=gpurun_out/knobs
mkdir -p $O
for E in "X=0" "HIP_FORCE_DEV_KERNARG=1" "HIP_FORCE_DEV_KERNARG=0" "ROC_USE_FGS_KERNARG=0" "ROC_USE_FGS_KERNARG=1" \
         "AMD_DIRECT_DISPATCH=0" "ROC_SYSTEM_SCOPE_SIGNAL=0" "DEBUG_CLR_KERNARG_HDP_FLUSH_WA=0" "ROC_SKIP_KERNEL_ARG_COPY=1" \
         "GPU_FLUSH_ON_EXECUTION=0"; do
  echo "$E: $(env $E timeout -k 5 60 tools/dispatch_cost q 2>&1 | tail -1)" | tee -a $O/knobs.txt
done
for E in "X=0" "HIP_FORCE_DEV_KERNARG=1" "ROC_USE_FGS_KERNARG=0" "AMD_DIRECT_DISPATCH=0"; do
  env $E timeout -k 10 120 python bench.py --workload invmgmt_lostsales --no-cpu-baseline --no-rollout-line > $O/ls_$E.json 2>$O/ls_$E.err || { tail $O/ls_$E.err; exit 1; }
  echo "$E lostsales step: $(python -c "import json; d=json.loads(open('$O/ls_$E.json').read().strip().splitlines()[-1]); print(round(d['value']/1e9,3), round(d['roofline']['kernel_ms_mean']*1e3,3))")" | tee -a $O/knobs.txt
done
