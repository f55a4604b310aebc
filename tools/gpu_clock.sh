#!/bin/bash
# Effective shader clock of the dominant kernel per case (GRBM_GUI_ACTIVE / 8 XCDs / kernel time,
# MI355X_MICROARCH.md "DVFS give-back"): one --pmc pass with the kernel trace per case.
#   CASES="v:kind ..." (DCT3D_ENC_VARIANT : bench --kind), BENCH_ARGS extra bench args.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/clock; mkdir -p $OUT
for cs in ${CASES:-1:ramp 1:uniform}; do
  v=${cs%%:*}; k=${cs##*:}
  DCT3D_ENC_VARIANT=$v timeout -k 10 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --kernel-trace -d $OUT/${v}_$k -o c --output-format csv -- \
    python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-ceiling --kind $k ${BENCH_ARGS} > $OUT/${v}_$k.log 2>&1
  rc=$?; echo "case $cs rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/${v}_$k.log; exit $rc; }
  python3 - "$OUT/${v}_$k" << 'PY'
import csv, glob, sys, collections
d = sys.argv[1]
cc = [r for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True) for r in csv.DictReader(open(f))]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for r in cc:
    k = r["Kernel_Name"]
    if "encode_kernel" in k or "decode_kernel" in k:
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        if "Start_Timestamp" in r and r.get("End_Timestamp"):
            acc[k]["ns"].append(float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))
for k, m in acc.items():
    g = sum(m["GRBM_GUI_ACTIVE"]) / len(m["GRBM_GUI_ACTIVE"])
    ns = sum(m["ns"]) / len(m["ns"]) if m["ns"] else float("nan")
    print(k[:60], "GRBM/8 %.3g cyc" % (g / 8), "kernel %.3f ms" % (ns / 1e6), "eff clock %.3f GHz" % (g / 8 / ns))
PY
done
