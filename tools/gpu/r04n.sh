#!/bin/bash
# Round 4, session n: the Newsvendor step's multiplication lookahead recomputing
# exp(-mu) instead of loading it -- Newsvendor GPU tests, A/B of the step
# against the previous kernel (ablate/NVOLD), FETCH pass.
set -u
OUT=gpurun_out/r04n
mkdir -p $OUT
export TMPDIR=/tmp
run() { echo "+ $*" >&2; "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" >&2; exit $rc; fi; }
run timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "newsvendor or nv_" > $OUT/pytest_nv.log 2>&1
tail -2 $OUT/pytest_nv.log
B="--workload newsvendor --no-cpu-baseline --no-rollout-line --no-graph-line"
for i in 1 2 3; do
  run timeout -k 10 120 python bench.py $B > $OUT/nv_step_new.$i.json 2>>$OUT/bench_err.log
  INVSIM_LIB=or-gym-inventory_amd/invsim/_lib/ablate/libinvsim_NVOLD.so run timeout -k 10 120 python bench.py $B > $OUT/nv_step_old.$i.json 2>>$OUT/bench_err.log
done
run timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- \
    python bench.py $B --steps 200 --warmup 20 > $OUT/pmc_fetch.log 2>&1
echo r04m done
