#!/bin/bash
# Round 6: what bounds net_rollq_kernel (ablation builds, timing only).
set -u
OUT=gpurun_out/r06g
mkdir -p $OUT
run() { echo "+ $*" >&2; "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" >&2; exit $rc; fi; }
B="--workload net_backlog --mode rollout --steps 1200 --warmup 60 --no-cpu-baseline"
L=or-gym-inventory_amd/invsim/_lib/abl6
for n in 4096 8192; do
  run timeout -k 10 120 python bench.py $B --n-envs $n > $OUT/prod_$n.json 2>$OUT/prod_$n.err
  for v in QNO_DRAW QNO_OBS QNO_OBS_DRAW QNO_DYN QONLY_DYN; do
    INVSIM_LIB=$L/libinvsim_$v.so run timeout -k 10 120 python bench.py $B --n-envs $n > $OUT/${v}_$n.json 2>$OUT/${v}_$n.err
  done
done
python - <<'PY'
import json
for n in (4096, 8192):
    row = []
    for v in ("prod", "QNO_DRAW", "QNO_OBS", "QNO_OBS_DRAW", "QNO_DYN", "QONLY_DYN"):
        d = json.loads(open(f"gpurun_out/r06g/{v}_{n}.json").read().splitlines()[-1])
        row.append(f'{v} {d["roofline"]["kernel_ms_mean"]*1e3:.1f}us')
    print(n, " | ".join(row))
PY
