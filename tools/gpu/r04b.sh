#!/bin/bash
# Round 4, session b: GPU suite on the staged NV rollout; per-wave timelines of
# the Newsvendor rollout and step (TIMING build); NV rollout A/B staged vs not;
# NV step XCD pairing A/B with PMC; VALU issue rates; closing-wait and warmup
# probes of the driver-style line.
set -u
OUT=gpurun_out/r04b
mkdir -p $OUT
export TMPDIR=/tmp
run() { echo "+ $*" >&2; "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" >&2; exit $rc; fi; }
run timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
tail -2 $OUT/pytest_gpu.log
INVSIM_LIB=or-gym-inventory_amd/invsim/_lib/ablate/libinvsim_TIMING.so run timeout -k 10 120 python tools/timing_nv_roll.py > $OUT/nv_roll_timeline.txt 2>&1
INVSIM_LIB=or-gym-inventory_amd/invsim/_lib/ablate/libinvsim_TIMING.so run timeout -k 10 120 python tools/timing_nv_step.py > $OUT/nv_step_timeline.txt 2>&1
R="--workload newsvendor --mode rollout --steps 1200 --warmup 60 --no-cpu-baseline"
for i in 1 2; do
  run timeout -k 10 120 python bench.py $R > $OUT/nv_roll_stage.$i.json 2>>$OUT/bench_err.log
  INVSIM_LIB=or-gym-inventory_amd/invsim/_lib/ablate/libinvsim_NOSTAGE.so run timeout -k 10 120 python bench.py $R > $OUT/nv_roll_nostage.$i.json 2>>$OUT/bench_err.log
done
for w in invmgmt_lostsales net_backlog; do
  for m in rollout policy; do
    R="--workload $w --mode $m --steps 1200 --warmup 60 --no-cpu-baseline"
    for i in 1 2; do
      run timeout -k 10 120 python bench.py $R > $OUT/${w}_${m}_stage.$i.json 2>>$OUT/bench_err.log
      INVSIM_LIB=or-gym-inventory_amd/invsim/_lib/ablate/libinvsim_NOSTAGE.so run timeout -k 10 120 python bench.py $R > $OUT/${w}_${m}_nostage.$i.json 2>>$OUT/bench_err.log
    done
  done
done
B="--workload newsvendor --no-cpu-baseline --no-rollout-line --no-graph-line"
for i in 1 2; do
  for x in 1 0; do
    INVSIM_NV_XCD=$x run timeout -k 10 120 python bench.py $B > $OUT/nv_xcd$x.$i.json 2>>$OUT/bench_err.log
  done
done
for x in 1 0; do
  INVSIM_NV_XCD=$x run timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch_xcd$x -o run -- \
      python bench.py $B --steps 200 --warmup 20 > $OUT/pmc_fetch_xcd$x.log 2>&1
done
run timeout -k 10 120 tools/valu_rates > $OUT/valu_rates.txt 2>&1
run timeout -k 10 120 python tools/sync_overhead.py --spin > $OUT/sync_overhead_spin.txt 2>&1
for w in 5 50 500; do
  run timeout -k 10 120 python bench.py --steps 20 --warmup $w --no-cpu-baseline --no-rollout-line --no-graph-line > $OUT/bench_w$w.json 2>>$OUT/bench_err.log
done
echo r04b done
