set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
T=gpurun_out/nvpmc
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU --output-format csv -d $T/a -o run -- python bench.py --workload newsvendor --mode rollout --steps 300 --warmup 60 --no-cpu-baseline > $T.a.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS --output-format csv -d $T/b -o run -- python bench.py --workload newsvendor --mode rollout --steps 300 --warmup 60 --no-cpu-baseline > $T.b.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU --output-format csv -d $T/c -o run -- python bench.py --steps 200 --warmup 20 --no-cpu-baseline > $T.c.log 2>&1 || exit 1
echo ok
