#!/bin/bash
# round 3 session c: new Net market / fast-stream tests, the round's bench +
# rocprofv3 kernel-trace / PMC (step and rollout) / SQ passes, and the PTRS
# margin statistics of the debug build over >= 1e8 draws per path
set -o pipefail
O=gpurun_out/r03c
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "market_samplers" tests/test_gpu_fast_stream.py -x -v --timeout 120 --timeout-method thread > $O/pytest_new.log 2>&1 || { tail -40 $O/pytest_new.log; exit 1; }
tail -2 $O/pytest_new.log
INVSIM_LIB=or-gym-inventory_amd/invsim/_lib/debug/libinvsim_ptrs_stats.so timeout -k 10 400 python tools/ptrs_margin.py > $O/ptrs_margin.json 2> $O/ptrs_margin.err || { tail -20 $O/ptrs_margin.err; exit 1; }
tail -c 600 $O/ptrs_margin.json
bash tools/gpu_round.sh r03c bench prof sq || exit 1
