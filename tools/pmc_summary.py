"""Summarise rocprofv3 --pmc counter_collection CSVs: average counter value per launch per kernel.

usage: python tools/pmc_summary.py out.csv a_counter_collection.csv [b_counter_collection.csv ...]
FETCH_SIZE / WRITE_SIZE are in KB (gfx950: FETCH_SIZE reads 1/2 of a wide coalesced stream, see
MI355X_MICROARCH.md §HBM -- the correction is applied where the numbers are used, not here)."""
import collections, csv, sys

acc = collections.defaultdict(list)
for f in sys.argv[2:]:
    for r in csv.DictReader(open(f)):
        acc[(r["Kernel_Name"], r["Counter_Name"])].append(float(r["Counter_Value"]))
with open(sys.argv[1], "w", newline="") as fo:
    w = csv.writer(fo)
    w.writerow(["kernel", "counter", "launches", "avg_per_launch_raw", "unit_note"])
    for (k, c), v in sorted(acc.items(), key=lambda x: (x[0][1], x[0][0])):
        if k.startswith(("__amd", "void at::")):
            continue
        w.writerow([k, c, len(v), round(sum(v) / len(v), 1), "KB" if c.endswith("_SIZE") else ""])
