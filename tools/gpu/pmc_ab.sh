set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
A=or-gym-inventory_amd/invsim/_lib/ablate
for L in cur $A/libinvsim_OLD.so; do
  P=or-gym-inventory_amd/invsim/_lib/libinvsim.so; [ $L != cur ] && P=$L
  T=gpurun_out/pmcab_$(basename $L .so)
  INVSIM_LIB=$P timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $T/trace -o run -- python bench.py --steps 300 --warmup 20 --no-cpu-baseline > $T.trace.log 2>&1 || exit 1
  INVSIM_LIB=$P timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $T/fetch -o run -- python bench.py --steps 100 --warmup 20 --no-cpu-baseline > $T.fetch.log 2>&1 || exit 1
  INVSIM_LIB=$P timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $T/write -o run -- python bench.py --steps 100 --warmup 20 --no-cpu-baseline > $T.write.log 2>&1 || exit 1
  INVSIM_LIB=$P timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $T/hit -o run -- python bench.py --steps 100 --warmup 20 --no-cpu-baseline > $T.hit.log 2>&1 || exit 1
done
echo ok
