#!/bin/bash
set -u
OUT=gpurun_out/net3; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "net" > $OUT/pytest_net.log 2>&1 || { tail -30 $OUT/pytest_net.log; exit 1; }
tail -1 $OUT/pytest_net.log
L=or-gym-inventory_amd/invsim/_lib/abl_tmp
bash tools/ab.sh net_backlog rollout cur $L/lib_ABL_ROLL_NO_STORE.so $L/lib_ABL_R3_NO_OBS.so $L/lib_ABL_ROLL_NO_DRAW.so
