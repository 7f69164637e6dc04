#!/bin/bash
# Round 6: what bounds the NetInvMgmt K=30 rollout at small shards (4 096 /
# 8 192 / 32 768 envs): the product kernel against ablation builds without the
# demand draws, without the obs wave's work, without both, without the tile
# stores (results wrong by construction; timing only).
set -u
OUT=gpurun_out/r06e
mkdir -p $OUT
run() { echo "+ $*" >&2; "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" >&2; exit $rc; fi; }
B="--workload net_backlog --mode rollout --steps 1200 --warmup 60 --no-cpu-baseline"
L=or-gym-inventory_amd/invsim/_lib/abl6
for n in 4096 8192 32768; do
  run timeout -k 10 120 python bench.py $B --n-envs $n > $OUT/prod_$n.json 2>$OUT/prod_$n.err
  for v in ROLL_NO_DRAW NET_NO_OBS NET_NO_OBS_DRAW ROLL_NO_STORE; do
    INVSIM_LIB=$L/libinvsim_$v.so run timeout -k 10 120 python bench.py $B --n-envs $n > $OUT/${v}_$n.json 2>$OUT/${v}_$n.err
  done
done
python - <<'PY'
import json
for n in (4096, 8192, 32768):
    row = []
    for v in ("prod", "ROLL_NO_DRAW", "NET_NO_OBS", "NET_NO_OBS_DRAW", "ROLL_NO_STORE"):
        d = json.loads(open(f"gpurun_out/r06e/{v}_{n}.json").read().splitlines()[-1])
        row.append(f'{v} {d["roofline"]["kernel_ms_mean"]*1e3:.1f}us')
    print(n, " | ".join(row))
PY
