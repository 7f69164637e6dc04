"""Summarise one tools/gpu_round.sh profile directory into profiles/<round>/pmc_<workload>.json.

  python tools/pmc_summary.py PROFDIR WORKLOAD KERNEL_SUBSTR OUT.json [step|rollout]

(rollout: the pmc_fetch_roll / pmc_write_roll passes and trace_roll stats of
`bench.py --mode rollout`, K = 30 steps per launch)

PROFDIR holds rocprofv3 outputs of `bench.py --workload WORKLOAD`:
trace/run_kernel_stats.csv (--kernel-trace --stats) and separate
pmc_fetch / pmc_write passes (run_counter_collection.csv).  HBM bytes per
launch = 2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes), with the factor 2 from
the MI355X calibration in profiles/r01/pmc_calib_*.json (tools/pmc_calib.hip:
FETCH_SIZE reports half the bytes of 8-B and 16-B/lane streaming reads).
"""
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import WORKLOADS  # noqa: E402


def counter_mean(path, name, kern):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if r["Counter_Name"] == name and kern in r["Kernel_Name"]]
    meta = None
    for r in csv.DictReader(open(path)):
        if kern in r["Kernel_Name"]:
            meta = {k: r[k] for k in ("Kernel_Name", "Grid_Size", "Workgroup_Size", "LDS_Block_Size",
                                      "Scratch_Size", "VGPR_Count", "Accum_VGPR_Count", "SGPR_Count")}
            break
    return (sum(vals) / len(vals) if vals else None), len(vals), meta


def main():
    prof, wl_name, kern, out = sys.argv[1:5]
    mode = sys.argv[5] if len(sys.argv) > 5 else "step"
    sfx, K = {"step": ("", 1), "rollout": ("_roll", 30), "policy": ("_pol", 30)}[mode]
    wl = WORKLOADS[wl_name]
    fetch, nf, meta = counter_mean(os.path.join(prof, "pmc_fetch" + sfx, "run_counter_collection.csv"),
                                   "FETCH_SIZE", kern)
    write, nw, _ = counter_mean(os.path.join(prof, "pmc_write" + sfx, "run_counter_collection.csv"),
                                "WRITE_SIZE", kern)
    stats = [r for r in csv.DictReader(open(os.path.join(prof, "trace" + sfx, "run_kernel_stats.csv")))
             if kern in r["Name"]]
    st = max(stats, key=lambda r: int(r["Calls"])) if stats else None
    B = wl["B_io"] + wl["B_state"] if K == 1 else wl["B_io"] + wl["B_state_rollout"] / K
    if mode == "policy":   # as bench.py: no action input, per-env metric sums once per launch
        md = {"invmgmt_backlog": 6, "invmgmt_lostsales": 6, "newsvendor": 2, "net_backlog": 11}[wl_name]
        B += -wl["B_act"] + 16 * md / K
    alg = B * wl["n"] * K
    hbm = 2.0 * fetch * 1024 + write * 1024 if fetch is not None and write is not None else None
    rec = {
        "kernel": f"{st['Name'] if st else kern} ({wl['desc']}, {mode}" + (f" K={K})" if K > 1 else ")"),
        "command": f"rocprofv3 --pmc FETCH_SIZE|WRITE_SIZE (separate passes) -- python bench.py "
                   f"--workload {wl_name}" + (f" --mode {mode} --steps 600 --warmup 60" if K > 1 else
                                              " --steps 200 --warmup 20") + " --no-cpu-baseline --no-rollout-line",
        "calibration": "tools/pmc_calib.hip on MI355X: FETCH_SIZE = 0.500 x bytes for 8-B and 16-B/lane "
                       "streaming reads -> x2; WRITE_SIZE = 1.000 x bytes",
        "FETCH_SIZE_KiB_mean": fetch, "FETCH_SIZE_dispatches": nf,
        "WRITE_SIZE_KiB_mean": write, "WRITE_SIZE_dispatches": nw,
        "hbm_bytes_per_launch": hbm,
        "algorithmic_bytes_per_launch": alg,
        "traffic_over_algorithmic": hbm / alg if hbm else None,
        "rocprof_kernel_ns_mean": float(st["AverageNs"]) if st else None,
        "rocprof_dispatches": int(st["Calls"]) if st else None,
        "achieved_GBps_rocprof": alg / float(st["AverageNs"]) if st else None,
        "launch": meta,
    }
    with open(out, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
