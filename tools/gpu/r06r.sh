#!/bin/bash
# Round 6: the 2-role InvMgmt rollout as back-to-back launches of at most
# INVSIM_IM_ROLL_SUB envs: parity, then K = 30 rollouts at 65 536 - 1 048 576
# envs, one launch (0) against sub-launches, alternating.
set -u
OUT=gpurun_out/r06r
mkdir -p $OUT
run() { echo "+ $*" >&2; "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" >&2; exit $rc; fi; }
run timeout -k 10 300 python -u -m pytest tests/test_gpu_roll_sub.py tests/test_gpu_episode_sink.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
tail -1 $OUT/pytest.log
B="--workload invmgmt_backlog --mode rollout --warmup 60 --no-cpu-baseline --no-config-lines --no-graph-line"
for i in 1 2; do
  for n in 65536 262144 1048576; do
    st=1200; [ $n = 1048576 ] && st=600
    for sub in 0 65536 131072; do
      [ $n = 65536 ] && [ $sub != 0 ] && sub=16384
      INVSIM_IM_ROLL_SUB=$sub run timeout -k 10 150 python bench.py $B --steps $st --n-envs $n > $OUT/n${n}_s${sub}_$i.json 2>$OUT/n${n}_s${sub}_$i.err
    done
  done
done
python - <<'PY'
import glob, json, re
rows = {}
for f in sorted(glob.glob("gpurun_out/r06r/n*_s*_*.json")):
    n, sub, i = re.match(r".*/n(\d+)_s(\d+)_(\d+).json", f).groups()
    d = json.loads(open(f).read().splitlines()[-1])
    rows.setdefault((int(n), int(sub)), []).append(f'{d["value"]/1e9:.2f}G {d["roofline"]["kernel_ms_mean"]*1e3:.0f}us f={d["roofline"]["frac"]:.3f}')
for k in sorted(rows):
    print(k, " | ".join(rows[k]))
PY
