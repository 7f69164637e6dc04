"""Tables of tools/measure_r05.sh outputs (profiling aid).

  python tools/sweep_summary.py gpurun_out/meas_r05 profiles/r05

sweep/n<N>/  ->  <out>/batch_sweep/table.md + table.json: the InvMgmt Backlog step
  and K=30 rollout at each batch size, with
  * the bench line's event-timed kernel time and algorithmic frac,
  * rocprofv3's per-kernel mean (kernel trace) and the frac on it,
  * HBM bytes per launch from FETCH_SIZE x 2 + WRITE_SIZE (separate passes,
    MI355X_MICROARCH.md's gfx950 correction) and the rate they move at
    (counter bytes / rocprof mean), i.e. the HBM-only fraction once the working
    set no longer fits the 256 MiB Infinity Cache.
strong/      ->  <out>/strong/table.md + table.json: per-rank sizes of configs 4
  and 5 (eager step, StepGraph replay, fused K=30 rollout) and the projected
  1->8 strong-scaling efficiency of config 5 (32 768 envs split over n ranks) and
  weak-scaling efficiency (fixed envs per rank).
"""
import csv
import glob
import json
import os
import re
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import HBM_PEAK_GBS, WORKLOADS  # noqa: E402


ROLL_SUB = 65536   # envs per im_roll3_kernel launch (csrc kernels.hpp im_roll_sub)


def last_json(path):
    for line in reversed(open(path).read().strip().split("\n")):
        line = line.strip()
        if line.startswith("{"):
            return json.loads(line)
    raise ValueError(f"no JSON line in {path}")


def stats_rows(d):
    f = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
    return list(csv.DictReader(open(f[0]))) if f else []


def main_kernel(rows, pat):
    rows = [r for r in rows if re.search(pat, r["Name"])]
    return max(rows, key=lambda r: float(r["TotalDurationNs"])) if rows else None


def counter(d, name, kern_name):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        return None
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(f[0]))
            if r["Counter_Name"] == name and r["Kernel_Name"] == kern_name]
    return sum(vals) / len(vals) if vals else None


def sweep(meas, out):
    res = []
    for d in sorted(glob.glob(os.path.join(meas, "sweep", "n*")), key=lambda p: int(p.rsplit("n", 1)[1])):
        n = int(d.rsplit("n", 1)[1])
        b = last_json(os.path.join(d, "bench.json"))
        wl = WORKLOADS["invmgmt_backlog"]
        for mode, sfx, pat, K in (("step", "", r"im_split_kernel", 1), ("rollout", "_roll", r"im_roll3o?_kernel", 30)):
            line = b if mode == "step" else b["rollout"]
            rf = line["roofline"]
            k = main_kernel(stats_rows(os.path.join(d, "trace" + sfx)), pat)
            kname = k["Name"] if k else None
            fetch = counter(os.path.join(d, "pmc_fetch" + sfx), "FETCH_SIZE", kname)
            write = counter(os.path.join(d, "pmc_write" + sfx), "WRITE_SIZE", kname)
            B = wl["B_io"] + (wl["B_state"] if K == 1 else wl["B_state_rollout"] / K)
            # per dispatch: since round 6 a rollout past 65 536 envs is back-to-back
            # launches of 65 536 envs (INVSIM_IM_ROLL_SUB's default), and rocprofv3 /
            # the counters report per launch
            alg = B * (n if K == 1 else min(n, ROLL_SUB)) * K
            ns = float(k["AverageNs"]) if k else None
            hbm = 2.0 * fetch * 1024 + write * 1024 if fetch is not None and write is not None else None
            res.append({
                "envs": n, "mode": mode + (f" K={K}" if K > 1 else ""), "kernel": kname,
                "env_steps_per_s": line["value"],
                "state_MiB": n * (wl["B_state"] if K == 1 else wl["B_state_rollout"]) / 2**20,
                "alg_bytes_per_launch": alg,
                "event_us": rf["kernel_ms_mean"] * 1e3, "frac_event": rf["frac_kernel"],
                "rocprof_us": ns / 1e3 if ns else None, "rocprof_calls": int(k["Calls"]) if k else None,
                "frac_rocprof": alg / ns / HBM_PEAK_GBS if ns else None,
                "fetch_bytes": 2.0 * fetch * 1024 if fetch is not None else None,
                "write_bytes": write * 1024 if write is not None else None,
                "hbm_bytes_per_launch": hbm,
                "traffic_over_alg": hbm / alg if hbm else None,
                "hbm_GBps": hbm / ns if hbm and ns else None,
                "frac_hbm_counters": hbm / ns / HBM_PEAK_GBS if hbm and ns else None,
            })
    os.makedirs(os.path.join(out, "batch_sweep"), exist_ok=True)
    json.dump(res, open(os.path.join(out, "batch_sweep", "table.json"), "w"), indent=1)
    L = ["| envs | mode | state MiB | env-steps/s | event µs | frac (event) | rocprof µs | frac (rocprof) "
         "| HBM B/launch (counters) | traffic / alg. | counter GB/s | HBM frac (counters) |",
         "|---|---|---|---|---|---|---|---|---|---|---|---|"]
    f = lambda x, p=3: "—" if x is None else f"{x:.{p}f}"  # noqa: E731
    for r in res:
        L.append(f"| {r['envs']:,} | {r['mode']} | {r['state_MiB']:.0f} | {r['env_steps_per_s'] / 1e9:.2f} G "
                 f"| {f(r['event_us'], 2)} | {f(r['frac_event'])} | {f(r['rocprof_us'], 2)} | {f(r['frac_rocprof'])} "
                 f"| {f(r['hbm_bytes_per_launch'] and r['hbm_bytes_per_launch'] / 1e6, 1)} MB "
                 f"| {f(r['traffic_over_alg'], 2)} | {f(r['hbm_GBps'], 0)} | {f(r['frac_hbm_counters'])} |")
    open(os.path.join(out, "batch_sweep", "table.md"), "w").write("\n".join(L) + "\n")
    for d in glob.glob(os.path.join(meas, "sweep", "n*")):
        for sub in ("trace", "trace_roll"):
            for src in glob.glob(os.path.join(d, sub, "**", "*kernel_stats.csv"), recursive=True):
                shutil.copy(src, os.path.join(out, "batch_sweep", f"{os.path.basename(d)}_{sub}_kernel_stats.csv"))
        shutil.copy(os.path.join(d, "bench.json"), os.path.join(out, "batch_sweep", f"{os.path.basename(d)}_bench.json"))
    print("\n".join(L))


def strong(meas, out):
    res = {}
    for p in sorted(glob.glob(os.path.join(meas, "strong", "*_*.json"))):
        m = re.match(r"(.+)_(\d+)\.json$", os.path.basename(p))
        w, n = m.group(1), int(m.group(2))
        b = last_json(p)
        k = main_kernel(stats_rows(os.path.join(meas, "strong", f"trace_{w}_{n}")), r"step|split")
        res[(w, n)] = {
            "workload": w, "envs": n,
            "step": b["value"], "step_ms": b["ms_per_step"], "step_event_us": b["roofline"]["kernel_ms_mean"] * 1e3,
            "step_kernel": k["Name"] if k else None, "step_rocprof_us": float(k["AverageNs"]) / 1e3 if k else None,
            "graph": b["graph"]["value"], "graph_ms": b["graph"]["ms_per_step"],
            "rollout": b["rollout"]["value"], "rollout_ms_per_launch": b["rollout"]["ms_per_launch"],
        }
    rows = sorted(res.values(), key=lambda r: (r["workload"], -r["envs"]))
    L = ["| workload | envs per rank | eager step env-steps/s | µs/step (wall) | step kernel µs (events) "
         "| StepGraph replay env-steps/s | K=30 rollout env-steps/s |", "|---|---|---|---|---|---|---|"]
    for r in rows:
        L.append(f"| {r['workload']} | {r['envs']:,} | {r['step'] / 1e9:.2f} G | {r['step_ms'] * 1e3:.2f} "
                 f"| {r['step_event_us']:.2f} | {r['graph'] / 1e9:.2f} G | {r['rollout'] / 1e9:.2f} G |")
    proj = []
    base = res.get(("net_backlog", 32768))
    if base:
        L += ["", "Config 5 (NetInvMgmt Backlog, 32 768 envs GLOBAL) split over n ranks, projected from the "
              "1-GPU rows (each rank runs its share; efficiency = speed-up / n):", "",
              "| ranks | envs per rank | mode | projected env-steps/s (all ranks) | speed-up | strong efficiency |",
              "|---|---|---|---|---|---|"]
        for nr in (1, 2, 4, 8):
            r = res.get(("net_backlog", 32768 // nr))
            if not r:
                continue
            for mode in ("step", "graph", "rollout"):
                tot = r[mode] * nr
                sp = tot / base[mode]
                proj.append({"ranks": nr, "envs_per_rank": 32768 // nr, "mode": mode, "value": tot,
                             "speedup": sp, "efficiency": sp / nr})
                L.append(f"| {nr} | {32768 // nr:,} | {mode} | {tot / 1e9:.2f} G | {sp:.2f} | {sp / nr:.2f} |")
    os.makedirs(os.path.join(out, "strong"), exist_ok=True)
    json.dump({"rows": rows, "config5_strong_projection": proj},
              open(os.path.join(out, "strong", "table.json"), "w"), indent=1)
    open(os.path.join(out, "strong", "table.md"), "w").write("\n".join(L) + "\n")
    for p in glob.glob(os.path.join(meas, "strong", "*.json")):
        shutil.copy(p, os.path.join(out, "strong", os.path.basename(p)))
    for p in glob.glob(os.path.join(meas, "strong", "trace_*", "**", "*kernel_stats.csv"), recursive=True):
        tag = p.split(os.sep + "strong" + os.sep)[1].split(os.sep)[0]
        shutil.copy(p, os.path.join(out, "strong", f"{tag}_kernel_stats.csv"))
    print("\n".join(L))


if __name__ == "__main__":
    meas, out = sys.argv[1], sys.argv[2]
    if os.path.isdir(os.path.join(meas, "sweep")):
        sweep(meas, out)
    if os.path.isdir(os.path.join(meas, "strong")):
        strong(meas, out)
