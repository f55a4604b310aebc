"""Per-kernel averages of a rocprofv3 --pmc run (counter_collection.csv files under a directory), as
profiles/pmc/<config>.csv rows: kernel,counter,launches,avg_per_launch_raw,unit_note (the counters' raw
units; bench.py pmc_traffic reads FETCH_SIZE / WRITE_SIZE in KB).  Run locally on the gpurun_out/ copy
(gpurun merges only gpurun_out/ back).
    python tools/pmc_summary.py <out.csv> <dir> [<dir> ...]"""
import collections
import csv
import glob
import os
import sys


def main():
    out, dirs = sys.argv[1], sys.argv[2:]
    acc = collections.defaultdict(list)  # (kernel, counter) -> values per dispatch
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            per = collections.defaultdict(float)  # (dispatch, kernel, counter) -> summed over dimensions
            for r in csv.DictReader(open(f)):
                per[(r.get("Dispatch_Id") or r.get("Correlation_Id"), r["Kernel_Name"], r["Counter_Name"])] += float(r["Counter_Value"])
            for (_, k, c), v in per.items():
                acc[(k, c)].append(v)
    with open(out, "w", newline="") as fo:
        w = csv.writer(fo)
        w.writerow(["kernel", "counter", "launches", "avg_per_launch_raw", "unit_note"])
        for (k, c), vs in sorted(acc.items()):
            if "dct3d::" not in k:  # the library's kernels only (not torch's bench-side helpers)
                continue
            w.writerow([k, c, len(vs), round(sum(vs) / len(vs), 1), "KB" if c in ("FETCH_SIZE", "WRITE_SIZE") else "raw"])


if __name__ == "__main__":
    main()
