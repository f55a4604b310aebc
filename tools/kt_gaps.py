#!/usr/bin/env python3
"""Consecutive dispatches of one kernel in a rocprofv3 --kernel-trace CSV: duration of each and the gap
from the previous dispatch's end (any kernel) to its start, so per-launch fixed costs show up.

  python3 tools/kt_gaps.py gpurun_out/kt/sep encode16_kernel [last N]
"""
import csv
import glob
import os
import sys


def main():
    root, name = sys.argv[1], sys.argv[2]
    last = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    files = glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True)
    rows = []
    for f in files:
        rows += list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    prev_end = None
    out = []
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if name in r["Kernel_Name"]:
            out.append((s, e, None if prev_end is None else s - prev_end))
        prev_end = e if prev_end is None else max(prev_end, e)
    out = out[-last:]
    durs = [(e - s) / 1e3 for s, e, _ in out]
    gaps = [g / 1e3 for _, _, g in out if g is not None]
    print(f"{name}: {len(out)} dispatches; duration us: mean {sum(durs) / len(durs):.1f} min {min(durs):.1f} "
          f"max {max(durs):.1f}; gap before us: mean {sum(gaps) / max(1, len(gaps)):.1f} "
          f"min {min(gaps) if gaps else 0:.1f} max {max(gaps) if gaps else 0:.1f}")
    print(" ".join(f"{d:.0f}/{g / 1e3 if g is not None else 0:.0f}" for (s, e, g), d in zip(out, durs)))


if __name__ == "__main__":
    main()
