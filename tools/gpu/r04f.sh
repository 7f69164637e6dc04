#!/bin/bash
# Round 4, session f: the Newsvendor lookahead reading only its sampler
# branch's constants (GPU tests, step bench, FETCH/WRITE passes); the 4-wave
# rollout timeline with loop-trip counts (ablate/TIMING).
set -u
OUT=gpurun_out/r04f
mkdir -p $OUT
export TMPDIR=/tmp
run() { echo "+ $*" >&2; "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" >&2; exit $rc; fi; }
run timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "newsvendor or nv_" > $OUT/pytest_nv.log 2>&1
tail -2 $OUT/pytest_nv.log
B="--workload newsvendor --no-cpu-baseline --no-rollout-line --no-graph-line"
for i in 1 2; do
  run timeout -k 10 120 python bench.py $B > $OUT/nv_step.$i.json 2>>$OUT/bench_err.log
done
run timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- \
    python bench.py $B --steps 200 --warmup 20 > $OUT/pmc_fetch.log 2>&1
run timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- \
    python bench.py $B --steps 200 --warmup 20 > $OUT/pmc_write.log 2>&1
INVSIM_LIB=or-gym-inventory_amd/invsim/_lib/ablate/libinvsim_TIMING.so run timeout -k 10 120 python tools/timing_nv_roll.py 4 > $OUT/nv_roll_timeline.txt 2>&1
echo r04f done
