#!/bin/bash
# Round 6: the Newsvendor PTRS straggler assist: parity, then the rollout
# (and policy rollout) with INVSIM_NV_TAIL=1 / 0, interleaved, three runs each.
set -u
OUT=gpurun_out/r06i
mkdir -p $OUT
run() { echo "+ $*" >&2; "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" >&2; exit $rc; fi; }
run timeout -k 10 400 python -u -m pytest tests/test_gpu_nv_tail.py tests/test_gpu_long_draws.py -k "tail or newsvendor or nv" -x -v --timeout 120 --timeout-method thread > $OUT/pytest_tail.log 2>&1
tail -2 $OUT/pytest_tail.log
run timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "newsvendor or nv_" -x -q --timeout 120 --timeout-method thread > $OUT/pytest_nv.log 2>&1
tail -2 $OUT/pytest_nv.log
B="--workload newsvendor --steps 1200 --no-cpu-baseline"
for i in 1 2 3; do
  for tl in 1 0; do
    INVSIM_NV_TAIL=$tl run timeout -k 10 120 python bench.py $B --mode rollout > $OUT/roll_${tl}_$i.json 2>$OUT/roll_${tl}_$i.err
    INVSIM_NV_TAIL=$tl run timeout -k 10 120 python bench.py $B --mode policy > $OUT/pol_${tl}_$i.json 2>$OUT/pol_${tl}_$i.err
  done
done
python - <<'PY'
import json
for m in ("roll", "pol"):
    for tl in (1, 0):
        row = []
        for i in (1, 2, 3):
            d = json.loads(open(f"gpurun_out/r06i/{m}_{tl}_{i}.json").read().splitlines()[-1])
            row.append(f'{d["value"]/1e9:.2f}G {d["roofline"]["kernel_ms_mean"]*1e3:.2f}us')
        print(m, "tail" if tl else "plain", " | ".join(row))
PY
# the InvMgmt Backlog policy rollout with the sink and with the block fold
for i in 1 2; do
  for f in sink inline; do
    run timeout -k 10 120 python bench.py --workload invmgmt_backlog --mode policy --steps 1200 --no-cpu-baseline --fold $f > $OUT/impol_${f}_$i.json 2>$OUT/impol_${f}_$i.err
  done
done
python - <<'PY'
import json
for f in ("sink", "inline"):
    row = []
    for i in (1, 2):
        d = json.loads(open(f"gpurun_out/r06i/impol_{f}_{i}.json").read().splitlines()[-1])
        row.append(f'{d["value"]/1e9:.2f}G {d["roofline"]["kernel_ms_mean"]*1e3:.2f}us')
    print("im policy", f, " | ".join(row))
PY
