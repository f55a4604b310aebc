"""Markdown table of a tools/gpu_round.sh directory: per config the bench line (G cubes/s, ms per step,
the dominant kernel's events time, roofline frac) and the rocprofv3 average of its dominant kernel.
    python tools/round_table.py profiles/r06/final"""
import csv, glob, json, os, sys

NAMES = {"c2": "c2 encode 8×8×8 1080p ×128", "c2u": "c2 uniform-noise content", "c3": "c3 decode 8×8×8 1080p ×128",
         "c3u": "c3 uniform-noise content", "c4": "c4 encode 4K, one 64-stack job", "c5": "c5 encode 8×8×4 1080p ×128",
         "c6": "c6 decode 8×8×4 1080p ×128", "c7": "c7 raster → Exp-Golomb stream", "c8": "c8 Exp-Golomb stream → raster",
         "c8u": "c8 uniform-noise content", "c9": "c9 drop-in (A) forward f32", "c10": "c10 drop-in (A) inverse f32"}
d = sys.argv[1]
print("| config | G cubes/s | ms/step | kernel ms (events) | rocprof avg ms (dominant kernel) | roofline frac |")
print("|---|---|---|---|---|---|")
for c in NAMES:
    f = os.path.join(d, f"bench_{c}.json")
    if not os.path.exists(f):
        continue
    r = json.load(open(f))
    roof = r.get("roofline") or {}
    ks = os.path.join(d, f"kernel_stats_{c}.csv")
    top = ""
    if os.path.exists(ks):
        rows = [x for x in csv.DictReader(open(ks)) if "dct3d" in x["Name"] and "synth" not in x["Name"]]
        if rows:
            x = max(rows, key=lambda x: float(x["TotalDurationNs"]))
            top = f"{float(x['AverageNs']) / 1e6:.3f} ({x['Name'].replace('(anonymous namespace)::', '').split('(')[0].split('::')[-1]})"
    frac = roof.get("frac")
    print(f"| {NAMES[c]} | {r['value'] / 1e9:.3f} | {r['ms_per_step']:.3f} | {roof.get('kernel_ms', 0):.3f} | {top} | "
          f"{'**%.3f**' % frac if c in ('c2', 'c8') else '%.3f' % frac} |")
