#!/bin/bash
# GPU tests, then rollout A/B of the in-tree build against the library $1 (three rollout workloads).
set -u
OUT=gpurun_out/pair; mkdir -p $OUT
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for w in net_backlog invmgmt_lostsales invmgmt_backlog; do
  echo "== $w"; bash tools/ab.sh $w rollout cur $1 || exit 1
done
