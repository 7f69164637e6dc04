#!/bin/bash
# round 3 final session, part 2: rocprofv3 kernel stats, FETCH/WRITE PMC passes, Newsvendor SQ counters
set -o pipefail
bash tools/gpu_round.sh r03h prof sq || exit 1
