#!/bin/bash
# c8 (stream -> raster) A/B on one box: the Exp-Golomb GPU tests, then bench.py c8 lines of each variant
# interleaved over ROUNDS rounds (ramp, and uniform content with UNIFORM=1), then a rocprofv3 kernel trace
# of each variant.  A variant is "label|extra bench args" (e.g. an --opt knob); default: the build as is.
#   OUT=r04_c8ab ROUNDS=3 UNIFORM=1 tools/gpu_c8_ab.sh "cur|" "x|--opt eg_dec_groups=4"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-c8ab}
mkdir -p $O
[ $# -eq 0 ] && set -- "cur|"
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 400 python -u -m pytest tests/test_gpu_eg.py tests/test_gpu_eg_fused.py -m gpu -x -q --timeout 120 \
     --timeout-method thread > $O/pytest_eg.log 2>&1
  rc=$?; tail -3 $O/pytest_eg.log; [ $rc -ne 0 ] && { echo "pytest rc=$rc"; exit $rc; }
fi
args=()
for v in "$@"; do args+=("${v%%|*}|--config c8_decode_eg_1080p ${v#*|}"); done
if [ -n "$UNIFORM" ]; then for v in "$@"; do args+=("${v%%|*}u|--config c8_decode_eg_1080p --kind uniform ${v#*|}"); done; fi
OUT=${O#gpurun_out/} ROUNDS=${ROUNDS:-3} tools/ab_args.sh "${args[@]}" || exit $?
[ -n "$NO_PROF" ] && exit 0
for v in "$@"; do
  label=${v%%|*}; extra=${v#*|}
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_$label -o run --output-format csv -- \
     python3 bench.py --config c8_decode_eg_1080p --steps 20 --warmup 5 --no-cpu-baseline --no-ceiling $extra \
     > $O/prof_$label.log 2>&1 || { echo "rocprof $label failed"; tail -3 $O/prof_$label.log; exit 1; }
  f=$(find $O/prof_$label -name '*kernel_stats.csv' | head -1); cp "$f" $O/kernel_stats_c8_$label.csv
  python3 -c "
import csv
for r in csv.DictReader(open('$O/kernel_stats_c8_$label.csv')):
    if 'eg_' in r['Name'] or 'decode_eg' in r['Name']: print('$label', r['Name'][:60], round(float(r['AverageNs'])/1e3,1), 'us')"
done
exit 0
