"""CPU restatement (oracle/oracle.c) throughput for every bench workload on this
host: single thread and OpenMP over the host's cores (bench.py's cpu_baseline
leg).  Runs without a GPU; used to relate this container's CPU to the GPU box's.

  python tools/cpu_side_by_side.py [seconds-per-workload]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def main():
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 8.0
    out = {}
    for w in ("newsvendor", "invmgmt_backlog", "invmgmt_lostsales", "net_backlog"):
        r = bench.cpu_baseline(bench.WORKLOADS[w], secs)
        out[w] = {"threads": r["cores"], "value": r["value"], "single_thread": r["single_thread"]["value"],
                  "cpu_model": r["cpu_model"]}
        print(w, json.dumps(out[w]), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
