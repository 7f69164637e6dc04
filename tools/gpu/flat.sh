#!/bin/bash
# GPU tests, then rollout A/B: in-tree build against the library given as $1.
set -u
OUT=gpurun_out/flat; mkdir -p $OUT
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for w in invmgmt_backlog invmgmt_lostsales; do
  echo "== $w"; bash tools/ab.sh $w rollout cur $1 || exit 1
done
