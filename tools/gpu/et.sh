#!/bin/bash
# A/B: the InvMgmt split step with the obs tail stored early by the window wave (make early_tail)
set -o pipefail
mkdir -p gpurun_out/et
L=or-gym-inventory_amd/invsim/_lib/ab/libinvsim_ET.so
INVSIM_LIB=$L timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fast_stream.py tests/test_gpu_graphs.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/et/pytest.log 2>&1 || { tail -40 gpurun_out/et/pytest.log; exit 1; }
tail -2 gpurun_out/et/pytest.log
for w in invmgmt_backlog invmgmt_lostsales; do
  bash tools/ab.sh $w step cur $L | tee gpurun_out/et/ab_$w.txt
done
