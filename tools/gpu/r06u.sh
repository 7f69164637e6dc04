#!/bin/bash
# Round 6: the window-row split, RW = 4 / 5 (product) / 6 / 7 against 9 (the
# window wave loads all nine rows), three alternating runs each.
set -u
OUT=gpurun_out/r06u
mkdir -p $OUT
run() { echo "+ $*" >&2; "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" >&2; exit $rc; fi; }
K='invmgmt or InvManagement or sink or config4 or offset'
#run timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_episode_sink.py -x -q --timeout 120 --timeout-method thread -k "$K" > $OUT/pytest.log 2>&1
#
for i in 1 2 3; do
  for w in invmgmt_backlog invmgmt_lostsales; do
    for v in cur RW9 RW4 RW6 RW7; do
      P=or-gym-inventory_amd/invsim/_lib/libinvsim.so; [ $v != cur ] && P=or-gym-inventory_amd/invsim/_lib/old/libinvsim_$v.so
      INVSIM_LIB=$P run timeout -k 10 120 python bench.py --workload $w --steps 2000 --warmup 100 --no-cpu-baseline --no-config-lines --no-rollout-line --no-graph-line > $OUT/${w}_${v}_$i.json 2>$OUT/${w}_${v}_$i.err
    done
  done
done
python - <<'PY'
import json
for w in ("invmgmt_backlog", "invmgmt_lostsales"):
    for v in ("RW9", "RW4", "cur", "RW6", "RW7"):
        row = []
        for i in (1, 2, 3):
            d = json.loads(open(f"gpurun_out/r06u/{w}_{v}_{i}.json").read().splitlines()[-1])
            row.append(f'{d["roofline"]["kernel_ms_mean"]*1e3:.2f}us')
        print(w, v, " | ".join(row))
PY
