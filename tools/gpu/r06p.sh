#!/bin/bash
# Round 6: the one-barrier split step (cur) against the round-5 two-barrier step
# (old/libinvsim_DSYNC.so) under rocprofv3 kernel tracing (each dispatch timed
# alone), alternating, InvMgmt Backlog 65 536 and LostSales 32 768.
set -u
OUT=gpurun_out/r06p
mkdir -p $OUT
export TMPDIR=/tmp
run() { echo "+ $*" >&2; "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" >&2; exit $rc; fi; }
B="--steps 1000 --warmup 50 --no-cpu-baseline --no-rollout-line --no-graph-line --no-config-lines"
for i in 1 2; do
  for w in invmgmt_backlog invmgmt_lostsales; do
    for v in cur DSYNC; do
      P=or-gym-inventory_amd/invsim/_lib/libinvsim.so; [ $v != cur ] && P=or-gym-inventory_amd/invsim/_lib/old/libinvsim_$v.so
      INVSIM_LIB=$P run timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${w}_${v}_$i -o run -- \
          python bench.py --workload $w $B > $OUT/${w}_${v}_$i.log 2>&1
    done
  done
done
python - <<'PY'
import csv
for w in ("invmgmt_backlog", "invmgmt_lostsales"):
    for v in ("DSYNC", "cur"):
        row = []
        for i in (1, 2):
            for r in csv.DictReader(open(f"gpurun_out/r06p/{w}_{v}_{i}/run_kernel_stats.csv")):
                if "im_split_kernel" in r["Name"]:
                    row.append(f'{float(r["AverageNs"])/1e3:.2f}us')
        print(w, v, " | ".join(row))
PY
