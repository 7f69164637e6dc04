#!/bin/bash
# Round 6: im_split_kernel, early window-chunk stores (cur) against the one-
# barrier step (old/libinvsim_NOEARLY.so) and the round-5 two-barrier step
# (old/libinvsim_DSYNC.so): InvMgmt parity, then alternating bench runs.
set -u
OUT=gpurun_out/r06n
mkdir -p $OUT
run() { echo "+ $*" >&2; "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" >&2; exit $rc; fi; }
#run timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_episode_sink.py -x -q --timeout 120 --timeout-method thread -k "invmgmt or InvManagement or sink or config4 or offset" > $OUT/pytest.log 2>&1
#tail -2 $OUT/pytest.log
for i in 1 2; do
  for w in invmgmt_backlog invmgmt_lostsales; do
    for v in cur old/libinvsim_NOEARLY.so old/libinvsim_DSYNC.so; do
      P=or-gym-inventory_amd/invsim/_lib/libinvsim.so; [ $v != cur ] && P=or-gym-inventory_amd/invsim/_lib/$v
      tag=$(case $v in cur) echo early;; *NOEARLY*) echo dec;; *) echo dsync;; esac)
      INVSIM_LIB=$P run timeout -k 10 120 python bench.py --workload $w --steps 2000 --warmup 100 --no-cpu-baseline --no-config-lines > $OUT/${w}_${tag}_$i.json 2>$OUT/${w}_${tag}_$i.err
    done
  done
done
python - <<'PY'
import json
for w in ("invmgmt_backlog", "invmgmt_lostsales"):
    for tag in ("dsync", "dec", "early"):
        row = []
        for i in (1, 2):
            d = json.loads(open(f"gpurun_out/r06n/{w}_{tag}_{i}.json").read().splitlines()[-1])
            row.append(f'{d["value"]/1e9:.3f}G {d["roofline"]["kernel_ms_mean"]*1e3:.2f}us')
        print(w, tag, " | ".join(row))
PY
