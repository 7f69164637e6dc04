#!/bin/bash
# Round 6: what the split step's window loads cost (timing-only ablation
# builds, results wrong by construction): WNONE = no window loads,
# WNEW = nine rows all from the newest ring slot (written by the previous
# launch, other env groups of the same XCD), against the product build.
set -u
OUT=gpurun_out/r06q
mkdir -p $OUT
run() { echo "+ $*" >&2; "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" >&2; exit $rc; fi; }
for i in 1 2; do
  for w in invmgmt_backlog invmgmt_lostsales; do
    for v in cur WNONE WNEW; do
      P=or-gym-inventory_amd/invsim/_lib/libinvsim.so; [ $v != cur ] && P=or-gym-inventory_amd/invsim/_lib/old/libinvsim_$v.so
      INVSIM_LIB=$P run timeout -k 10 120 python bench.py --workload $w --steps 2000 --warmup 100 --no-cpu-baseline --no-config-lines --no-rollout-line --no-graph-line > $OUT/${w}_${v}_$i.json 2>$OUT/${w}_${v}_$i.err
    done
  done
done
python - <<'PY'
import json
for w in ("invmgmt_backlog", "invmgmt_lostsales"):
    for v in ("cur", "WNONE", "WNEW"):
        row = []
        for i in (1, 2):
            d = json.loads(open(f"gpurun_out/r06q/{w}_{v}_{i}.json").read().splitlines()[-1])
            row.append(f'{d["roofline"]["kernel_ms_mean"]*1e3:.2f}us')
        print(w, v, " | ".join(row))
PY
