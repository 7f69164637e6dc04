#!/bin/bash
# wave -> SIMD placement of multi-wave workgroups (tools/wave_placement)
set -o pipefail
O=gpurun_out/placement
mkdir -p $O
for cfg in "3 512 3" "2 768 2" "2 1024 2" "6 256 3" "4 256 2" "3 1024 3" "6 512 3"; do
  echo "== $cfg" >> $O/placement.txt
  timeout -k 5 30 tools/wave_placement $cfg >> $O/placement.txt 2>&1 || exit 1
done
cat $O/placement.txt
timeout -k 5 60 tools/dispatch_cost > $O/dispatch_cost.txt 2>&1 || exit 1
cat $O/dispatch_cost.txt
