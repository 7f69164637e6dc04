set -o pipefail
A=or-gym-inventory_amd/invsim/_lib/ablate
for rep in 1 2; do
for L in $A/libinvsim_OLD.so or-gym-inventory_amd/invsim/_lib/libinvsim.so $A/libinvsim_SS.so; do
  INVSIM_LIB=$L timeout -k 10 100 python bench.py --steps 6000 --warmup 200 --no-cpu-baseline > gpurun_out/ab.log 2>&1 || exit 1
  echo "$rep $(basename $L) $(tail -1 gpurun_out/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e9,3), round(d["roofline"]["kernel_ms_mean"]*1e3,3))')"
done; done
