"""Copy one tools/gpu_round.sh output (gpurun_out/round_TAG) into profiles/ROUND:
per-workload rocprofv3 kernel stats, the PMC summary JSON (tools/pmc_summary.py)
and the bench JSON lines, plus a markdown table of the lot.

  python tools/collect_round.py TAG [ROUND=r01]
"""
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ROLL_KERNELS = {"invmgmt_backlog": "im_roll3_kernel", "invmgmt_lostsales": "im_roll3o_kernel",
                "newsvendor": "nv_roll_kernel", "net_backlog": "net_roll3o_kernel"}
POL_KERNELS = {"invmgmt_backlog": "im_roll3_kernel", "invmgmt_lostsales": "im_roll3o_kernel",
               "newsvendor": "nv_roll_kernel", "net_backlog": "net_roll3o_kernel"}
KERNELS = {"invmgmt_backlog": "im_split_kernel", "invmgmt_lostsales": "im_split_kernel",
           "newsvendor": "nv_step1_kernel", "net_backlog": "net_step2_kernel"}


def last_json(path):
    if not os.path.exists(path):
        return None
    for line in reversed(open(path).read().splitlines()):
        if line.startswith("{"):
            return json.loads(line)
    return None


def kernel_avg_ns(csv_path, kern):
    """Average duration (ns) of the named kernel in a rocprofv3 kernel_stats.csv."""
    import csv
    if not os.path.exists(csv_path):
        return None
    for row in csv.DictReader(open(csv_path)):
        if kern in row["Name"]:
            return float(row["AverageNs"])
    return None


def median_trace(prof, wl, kern, dst):
    """gpu_round.sh trace3: three kernel-trace runs of the step bench (trace,
    trace_2, trace_3).  The run whose dominant-kernel mean is the median becomes
    trace/run_kernel_stats.csv (run 1's file is kept beside it as
    run_kernel_stats.run1.csv); the three means go to
    profiles/<round>/<workload>_step_trace_runs.json."""
    runs = [d for d in ("trace", "trace_2", "trace_3") if os.path.exists(os.path.join(prof, d, "run_kernel_stats.csv"))]
    if len(runs) < 3:
        return
    keep = os.path.join(prof, "trace", "run_kernel_stats.run1.csv")
    if not os.path.exists(keep):
        shutil.copy(os.path.join(prof, "trace", "run_kernel_stats.csv"), keep)
    paths = {d: keep if d == "trace" else os.path.join(prof, d, "run_kernel_stats.csv") for d in runs}
    ns = {d: kernel_avg_ns(p, kern) for d, p in paths.items()}
    order = sorted(runs, key=lambda d: ns[d])
    med = order[1]
    shutil.copy(paths[med], os.path.join(prof, "trace", "run_kernel_stats.csv"))
    with open(os.path.join(dst, f"{wl}_step_trace_runs.json"), "w") as f:
        json.dump({"kernel": kern, "mean_ns_per_run": ns, "kept": med,
                   "rule": "median of three rocprofv3 --kernel-trace --stats runs of the step bench"}, f, indent=1)


def issue_frac(src, wl, mode, kern_ms):
    """Newsvendor's issue-rate roofline from this round's SQ passes (bench.py
    _issue): VALU + SALU wave-instructions per launch over 1 024 SIMDs x the
    launch's cycles at 2.4 GHz / 2.2 cycles per instruction."""
    if wl != "newsvendor" or mode not in ("step", "rollout"):
        return " |"
    sq = os.path.join(ROOT, "profiles", "_sq_tmp.json")
    d = os.path.join(src, "sq_newsvendor")
    if not os.path.isdir(d):
        return " |"
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "sq_summary.py"), d, sq], check=True,
                   capture_output=True)
    c = json.load(open(sq))[mode]["counters_mean_per_dispatch"]
    os.remove(sq)
    insts = c["SQ_INSTS_VALU"] + c["SQ_INSTS_SALU"]
    return f" {insts / (1024 * kern_ms * 1e-3 * 2.4e9 / 2.2):.3f} |"


def main():
    tag = sys.argv[1]
    rnd = sys.argv[2] if len(sys.argv) > 2 else "r01"
    src = os.path.join(ROOT, "gpurun_out", f"round_{tag}")
    dst = os.path.join(ROOT, "profiles", rnd)
    os.makedirs(dst, exist_ok=True)
    rows = []
    for wl, kern in KERNELS.items():
        prof = os.path.join(src, f"prof_{wl}")
        if os.path.isdir(prof):
            median_trace(prof, wl, kern, dst)
            shutil.copy(os.path.join(prof, "trace", "run_kernel_stats.csv"),
                        os.path.join(dst, f"{wl}_step_kernel_stats.csv"))
            roll = os.path.join(prof, "trace_roll", "run_kernel_stats.csv")
            if os.path.exists(roll):
                shutil.copy(roll, os.path.join(dst, f"{wl}_rollout_kernel_stats.csv"))
            subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_summary.py"), prof, wl, kern,
                            os.path.join(dst, f"pmc_{wl}.json")], check=True, capture_output=True)
            if os.path.isdir(os.path.join(prof, "pmc_fetch_roll")):
                subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_summary.py"), prof, wl,
                                ROLL_KERNELS[wl], os.path.join(dst, f"pmc_{wl}_rollout.json"), "rollout"],
                               check=True, capture_output=True)
            if os.path.isdir(os.path.join(prof, "pmc_fetch_pol")):
                shutil.copy(os.path.join(prof, "trace_pol", "run_kernel_stats.csv"),
                            os.path.join(dst, f"{wl}_policy_kernel_stats.csv"))
                subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_summary.py"), prof, wl,
                                POL_KERNELS[wl], os.path.join(dst, f"pmc_{wl}_policy.json"), "policy"],
                               check=True, capture_output=True)
        for mode in ("step", "rollout", "policy"):
            b = last_json(os.path.join(src, f"bench_{wl}_{mode}.log"))
            if b is None:
                continue
            with open(os.path.join(dst, f"bench_{wl}_{mode}.json"), "w") as f:
                json.dump(b, f, indent=1)
            r = b["roofline"]
            pmc = os.path.join(dst, f"pmc_{wl}.json" if mode == "step" else f"pmc_{wl}_{mode}.json")
            pm = json.load(open(pmc)) if os.path.exists(pmc) else {}
            rp_ns = (pm.get("rocprof_kernel_ns_mean") if pm else None) or kernel_avg_ns(
                os.path.join(dst, f"{wl}_{mode}_kernel_stats.csv"),
                (KERNELS if mode == "step" else ROLL_KERNELS if mode == "rollout" else POL_KERNELS)[wl])
            alg = r["bytes_per_env_step"] * b["config"]["envs_per_gpu"] * (1 if mode == "step" else 30)
            rows.append(f"| {wl} | {mode} | {b['config']['envs_per_gpu']} | {b['value'] / 1e9:.3f} G | "
                        f"{r['kernel_ms_mean'] * 1e3:.2f} | {r['bytes_per_env_step']:.0f} | {r['achieved']:.0f} | "
                        f"{r['frac']:.3f} | "
                        + (f"{rp_ns / 1e3:.2f} | {alg / rp_ns / 8000.0:.3f} | " if rp_ns else "| | ")
                        + (f"{pm['traffic_over_algorithmic']:.2f} |" if pm and pm.get("traffic_over_algorithmic")
                           else " |")
                        + issue_frac(src, wl, mode, r["kernel_ms_mean"]))
    sq = os.path.join(src, "sq_newsvendor")
    if os.path.isdir(sq):
        subprocess.run([sys.executable, os.path.join(ROOT, "tools", "sq_summary.py"), sq,
                        os.path.join(dst, "sq_newsvendor.json")], check=True, capture_output=True)
    d = last_json(os.path.join(src, "bench_default.log"))
    if d:
        with open(os.path.join(dst, "bench_default.json"), "w") as f:
            json.dump(d, f, indent=1)
    with open(os.path.join(dst, "SUMMARY.md"), "w") as f:
        f.write(f"# Round {rnd} measurements (gpurun_out/round_{tag}, 1x MI355X)\n\n")
        f.write("| workload | mode | envs | env-steps/s | kernel µs/launch (events) | B/env-step | "
                "achieved GB/s | frac of 8 TB/s | rocprof µs/launch | frac on rocprof time | "
                "PMC traffic / algorithmic | issue frac |\n")
        f.write("|---|---|---|---|---|---|---|---|---|---|---|---|\n")
        f.write("\n".join(rows) + "\n")
    print(open(os.path.join(dst, "SUMMARY.md")).read())


if __name__ == "__main__":
    main()
