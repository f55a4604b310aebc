"""Print the per-kernel averages of kernel_stats_<label>_<round>.csv files under a gpurun_out directory
(tools/gpu_kstats.sh), with the bench line's ms per step from bench_<label>_<round>.json or the log.
    python tools/kstats_show.py gpurun_out/r06_walk [kernel regex]"""
import csv, glob, json, os, re, sys

d = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else "eg_|front"
for f in sorted(glob.glob(os.path.join(d, "kernel_stats_*.csv")), key=os.path.getmtime):
    tag = os.path.basename(f)[len("kernel_stats_"):-4]
    ms = None
    for src in (os.path.join(d, f"bench_{tag}.json"), os.path.join(d, f"prof_{tag}.log")):
        if os.path.exists(src):
            for line in open(src):
                if line.startswith('{"metric"'):
                    ms = json.loads(line)["ms_per_step"]
    parts = [f"{r['Name'].replace('(anonymous namespace)::', '').split('(')[0].split('::')[-1][:26]} {float(r['AverageNs']) / 1e3:.1f}"
             for r in csv.DictReader(open(f)) if float(r["Calls"]) > 10 and re.search(pat, r["Name"])]
    print(f"{tag:10s} ms/step {ms if ms is None else round(ms, 4)} | " + " | ".join(parts))
