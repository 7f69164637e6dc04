#!/bin/bash
# Round 6: the split step with the window rows shared between the waves
# (INVSIM_IM_SPLIT_RW: the window wave loads rows 0..RW-1, the dynamics wave
# the rest of the nine). Product RW = 5; A/B builds RW = 9 (window wave only,
# the previous kernel), 3 and 7. InvMgmt parity on the product and on RW = 3,
# then alternating bench runs.
set -u
OUT=gpurun_out/r06t
mkdir -p $OUT
run() { echo "+ $*" >&2; "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" >&2; exit $rc; fi; }
K='invmgmt or InvManagement or sink or config4 or offset'
run timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_episode_sink.py -x -q --timeout 120 --timeout-method thread -k "$K" > $OUT/pytest.log 2>&1
tail -1 $OUT/pytest.log
INVSIM_LIB=or-gym-inventory_amd/invsim/_lib/old/libinvsim_RW3.so run timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "$K" > $OUT/pytest_rw3.log 2>&1
tail -1 $OUT/pytest_rw3.log
for i in 1 2; do
  for w in invmgmt_backlog invmgmt_lostsales; do
    for v in cur RW9 RW3 RW7; do
      P=or-gym-inventory_amd/invsim/_lib/libinvsim.so; [ $v != cur ] && P=or-gym-inventory_amd/invsim/_lib/old/libinvsim_$v.so
      INVSIM_LIB=$P run timeout -k 10 120 python bench.py --workload $w --steps 2000 --warmup 100 --no-cpu-baseline --no-config-lines --no-rollout-line --no-graph-line > $OUT/${w}_${v}_$i.json 2>$OUT/${w}_${v}_$i.err
    done
  done
done
python - <<'PY'
import json
for w in ("invmgmt_backlog", "invmgmt_lostsales"):
    for v in ("RW9", "cur", "RW3", "RW7"):
        row = []
        for i in (1, 2):
            d = json.loads(open(f"gpurun_out/r06t/{w}_{v}_{i}.json").read().splitlines()[-1])
            row.append(f'{d["roofline"]["kernel_ms_mean"]*1e3:.2f}us')
        print(w, v, " | ".join(row))
PY
