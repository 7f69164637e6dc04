"""Summarise the SQ counter passes of tools/gpu_round.sh (part `sq`) into one
JSON: per kernel (nv_step1_kernel, nv_roll_kernel), the mean per dispatch of
every counter collected, plus derived issue figures.

  python tools/sq_summary.py gpurun_out/round_TAG/sq_newsvendor OUT.json

Derived (per dispatch): VALU instructions per wave; VALU busy share
SQ_ACTIVE_INST_VALU / SQ_BUSY_CYCLES (per-SIMD-cycle units differ by the SQ's
aggregation, so ratios between variants of one kernel are what to compare);
wait share SQ_WAIT_ANY / SQ_WAVE_CYCLES (waves parked on s_waitcnt / barrier)
and issue-stall share SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES.
"""
import csv
import glob
import json
import os
import sys

KERNELS = {"step": "nv_step1_kernel", "rollout": "nv_roll_kernel"}


def collect(path, kern):
    acc, n, meta = {}, {}, None
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if kern not in r["Kernel_Name"]:
                continue
            k = r["Counter_Name"]
            acc[k] = acc.get(k, 0.0) + float(r["Counter_Value"])
            n[k] = n.get(k, 0) + 1
            if meta is None:
                meta = {x: r.get(x) for x in ("Kernel_Name", "Grid_Size", "Workgroup_Size", "LDS_Block_Size",
                                              "Scratch_Size", "VGPR_Count", "Accum_VGPR_Count", "SGPR_Count")}
    # rows are per dispatch per counter (possibly per XCC/SE dimension): mean per dispatch
    disp = {}
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if kern in r["Kernel_Name"]:
                disp.setdefault(r["Counter_Name"], set()).add(r.get("Dispatch_Id") or r.get("Correlation_Id"))
    mean = {k: acc[k] / max(1, len(disp.get(k, ())) or n[k]) for k in acc}
    return mean, meta


def main():
    src, out = sys.argv[1:3]
    res = {}
    for m, kern in KERNELS.items():
        c = {}
        meta = None
        for part in ("a", "b"):
            mm, mt = collect(os.path.join(src, f"{m}.{part}"), kern)
            c.update(mm)
            meta = meta or mt
        d = {}
        if c.get("SQ_WAVES"):
            d["valu_insts_per_wave"] = c.get("SQ_INSTS_VALU", 0) / c["SQ_WAVES"]
            d["vmem_insts_per_wave"] = c.get("SQ_INSTS_VMEM", 0) / c["SQ_WAVES"]
            d["salu_insts_per_wave"] = c.get("SQ_INSTS_SALU", 0) / c["SQ_WAVES"]
        if c.get("SQ_BUSY_CYCLES"):
            d["active_valu_over_busy"] = c.get("SQ_ACTIVE_INST_VALU", 0) / c["SQ_BUSY_CYCLES"]
        if c.get("SQ_WAVE_CYCLES"):
            d["wait_any_over_wave_cycles"] = c.get("SQ_WAIT_ANY", 0) / c["SQ_WAVE_CYCLES"]
            d["wait_inst_any_over_wave_cycles"] = c.get("SQ_WAIT_INST_ANY", 0) / c["SQ_WAVE_CYCLES"]
            d["active_inst_any_over_wave_cycles"] = c.get("SQ_ACTIVE_INST_ANY", 0) / c["SQ_WAVE_CYCLES"]
        res[m] = {"kernel": kern, "counters_mean_per_dispatch": c, "derived": d, "launch": meta}
    res["command"] = ("rocprofv3 --pmc <8 SQ counters> and --pmc <4 SQ + 2 GRBM> (separate passes) -- python bench.py "
                      "--workload newsvendor [--mode rollout] --no-cpu-baseline --no-rollout-line")
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
