#!/bin/bash
# Round 6: net_rollq_kernel, branch-free dynamics: parity, then the roles alone
# (ablation builds, timing only) at 4 096 / 8 192 envs.
set -u
OUT=gpurun_out/r06h
mkdir -p $OUT
run() { echo "+ $*" >&2; "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" >&2; exit $rc; fi; }
run timeout -k 10 300 python -u -m pytest tests/test_gpu_net_small.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest_small.log 2>&1
tail -2 $OUT/pytest_small.log
B="--workload net_backlog --mode rollout --steps 1200 --warmup 60 --no-cpu-baseline"
L=or-gym-inventory_amd/invsim/_lib/abl6
for n in 4096 8192; do
  INVSIM_NET_ROLLQ_MAX_N=0 run timeout -k 10 120 python bench.py $B --n-envs $n > $OUT/roll3o_$n.json 2>$OUT/roll3o_$n.err
  run timeout -k 10 120 python bench.py $B --n-envs $n > $OUT/prod_$n.json 2>$OUT/prod_$n.err
  for v in QDEMAND_ONLY QOBS_ONLY QONLY_DYN QNOTHING; do
    INVSIM_LIB=$L/libinvsim_$v.so run timeout -k 10 120 python bench.py $B --n-envs $n > $OUT/${v}_$n.json 2>$OUT/${v}_$n.err
  done
done
python - <<'PY'
import json
for n in (4096, 8192):
    row = []
    for v in ("roll3o", "prod", "QDEMAND_ONLY", "QOBS_ONLY", "QONLY_DYN", "QNOTHING"):
        d = json.loads(open(f"gpurun_out/r06h/{v}_{n}.json").read().splitlines()[-1])
        row.append(f'{v} {d["roofline"]["kernel_ms_mean"]*1e3:.1f}us')
    print(n, " | ".join(row))
PY
