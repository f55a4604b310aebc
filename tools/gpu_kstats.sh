#!/bin/bash
# Kernel-stats A/B on one box: the GPU tests TESTS of the working tree (optional), then for each
# "label|dir|bench args" a rocprofv3 --kernel-trace --stats run of bench.py in dir (. or ab/<side>),
# printing the per-kernel average of the kernels matching KMATCH (default: Exp-Golomb kernels).
#   OUT=r06_x TESTS="tests/test_gpu_eg.py" tools/gpu_kstats.sh "cur|.|--config c8_decode_eg_1080p" \
#       "base|ab/base|--config c8_decode_eg_1080p"
# Any GPU fault / abort / timeout / segfault ends the script: nothing else runs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
ROOT=$(pwd)
O=gpurun_out/${OUT:-kst}
mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 ${PYTEST_TIMEOUT:-400} python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread \
     > $O/pytest.log 2>&1
  rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && { echo "pytest rc=$rc"; exit $rc; }
fi
for r in $(seq 1 ${ROUNDS:-1}); do
for v in "$@"; do
  IFS='|' read -r label dir args <<< "$v"
  (cd $dir && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $ROOT/$O/prof_${label}_$r -o run --output-format csv -- \
     python3 bench.py $args --steps 20 --warmup 5 --no-cpu-baseline --no-ceiling) > $O/prof_${label}_$r.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "rocprof $label rc=$rc"; tail -3 $O/prof_${label}_$r.log; exit $rc; }
  f=$(find $O/prof_${label}_$r -name '*kernel_stats.csv' | head -1); cp "$f" $O/kernel_stats_${label}_$r.csv
  [ -z "$KEEP_TRACE" ] && rm -rf $O/prof_${label}_$r  # the traces: 10+ MiB each (gpurun copies back <= 64 MiB)
  grep '^{"metric"' $O/prof_${label}_$r.log | tail -1 > $O/bench_${label}_$r.json
  python3 - "$O/kernel_stats_${label}_$r.csv" "$O/bench_${label}_$r.json" "$label" "${KMATCH:-eg_|front}" <<'PY'
import csv, json, re, sys
f, b, label, pat = sys.argv[1:5]
ms = json.load(open(b))["ms_per_step"]
parts = [f"{r['Name'].split('(')[0].split('::')[-1][:28]} {float(r['AverageNs'])/1e3:.1f}"
         for r in csv.DictReader(open(f)) if float(r["Calls"]) > 10 and re.search(pat, r["Name"])]
print(label, f"ms/step {ms:.4f} |", " | ".join(parts))
PY
done
done
exit 0
