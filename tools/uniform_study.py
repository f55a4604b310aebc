"""Ramp vs uniform-noise content, summarised (tools/gpu_uniform_study.sh output): per config the dominant
kernel's duration, effective shader clock (GRBM_GUI_ACTIVE / 8 XCDs / duration, medians over the last two
thirds of the launches) and SQ counters per wave.  One JSON object per config, then a markdown table.
    python tools/uniform_study.py gpurun_out [uniform] > profiles/r06/uniform/summary.md"""
import collections, csv, glob, json, os, statistics, sys

root = sys.argv[1]
tag = sys.argv[2] if len(sys.argv) > 2 else "uniform"
KERN = {"c2": "encode16_kernel", "c2u": "encode16_kernel", "c3": "decode_kernel<8", "c3u": "decode_kernel<8"}
rows = {}
for c, kname in KERN.items():
    d = os.path.join(root, tag, c)
    per = collections.defaultdict(dict)
    for r in csv.DictReader(open(glob.glob(os.path.join(d, "*counter_collection.csv"))[0])):
        if kname in r["Kernel_Name"]:
            k = r["Dispatch_Id"]
            per[k][r["Counter_Name"]] = per[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            per[k]["dur_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    launches = [per[k] for k in sorted(per, key=int)]
    late = launches[len(launches) // 3:]
    dur = statistics.median(x["dur_ns"] for x in late)
    clk = statistics.median(x["GRBM_GUI_ACTIVE"] / 8 / x["dur_ns"] for x in late)
    sq = collections.defaultdict(list)
    for f in glob.glob(os.path.join(root, f"sq_{tag}_{c}", "**", "*counter_collection.csv"), recursive=True):
        acc = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            if kname in r["Kernel_Name"]:
                acc[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        for (_, n), v in acc.items():
            sq[n].append(v)
    avg = {n: sum(v) / len(v) for n, v in sq.items()}
    waves = avg.get("SQ_WAVES", 1.0)
    rows[c] = {"kernel_ms": dur / 1e6, "clock_GHz": clk, "launches": len(launches),
               **{f"{n}_per_wave": v / waves for n, v in avg.items() if n not in ("SQ_WAVES", "GRBM_GUI_ACTIVE")},
               "waves": waves}
    print(json.dumps({"config": c, **{k: round(v, 4) for k, v in rows[c].items()}}))
keys = ["kernel_ms", "clock_GHz", "SQ_INSTS_VALU_per_wave", "SQ_INSTS_SALU_per_wave", "SQ_INSTS_LDS_per_wave",
        "SQ_INSTS_VMEM_RD_per_wave", "SQ_INSTS_VMEM_WR_per_wave", "SQ_WAIT_INST_ANY_per_wave", "SQ_WAVE_CYCLES_per_wave",
        "SQ_BUSY_CYCLES_per_wave"]
print("\n| | " + " | ".join(KERN) + " |\n|---|" + "---|" * len(KERN))
for k in keys:
    print(f"| {k} | " + " | ".join(f"{rows[c].get(k, float('nan')):.4g}" for c in KERN) + " |")
