#!/bin/bash
# One GPU session: kernel-trace stats + separate PMC passes for the bench workload,
# then bench lines for the other workloads/modes.  Usage: tools/gpu_profile.sh TAG [bench args...]
set -u
TAG=${1:-r01}; shift || true
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
run() { echo "+ $*"; "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
run timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python bench.py --steps 1000 --warmup 50 --no-cpu-baseline "$@"
run timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- \
    python bench.py --steps 200 --warmup 20 --no-cpu-baseline "$@"
run timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- \
    python bench.py --steps 200 --warmup 20 --no-cpu-baseline "$@"
echo "profile done"
