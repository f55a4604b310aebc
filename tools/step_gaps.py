#!/usr/bin/env python3
"""The dispatches of the last steps in a rocprofv3 --kernel-trace CSV: each one's duration and the idle gap
before it, so the launch overhead between a step's kernels shows up (a step ends with the kernel `last`).
skip: steps at the end of the trace to leave out -- bench.py's kernel-timing pass (its --steps steps after
the timed region) runs each launch between events, whose packets add gaps of their own.

  python3 tools/step_gaps.py gpurun_out/<dir> decode_eg_kernel [steps] [skip]
"""
import csv
import glob
import os
import sys


def main():
    root, last = sys.argv[1], sys.argv[2]
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    skip = int(sys.argv[4]) if len(sys.argv) > 4 else 0
    rows = []
    for f in glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(rows) if last in r["Kernel_Name"]]
    ends = ends[:len(ends) - skip] if skip else ends
    if len(ends) < steps + 1:
        sys.exit("not enough steps in the trace")
    first = ends[-steps - 1] + 1
    prev = int(rows[first - 1]["End_Timestamp"])
    busy = gap = 0.0
    for r in rows[first:ends[-1] + 1]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = r["Kernel_Name"].split("(")[0].split("::")[-1][:40]
        print(f"{name:40s} {(e - s) / 1e3:9.1f} us   gap before {(s - prev) / 1e3:6.1f} us")
        busy += (e - s) / 1e3
        gap += (s - prev) / 1e3
        prev = e
    print(f"per step: kernels {busy / steps:.1f} us, gaps {gap / steps:.1f} us")


if __name__ == "__main__":
    main()
