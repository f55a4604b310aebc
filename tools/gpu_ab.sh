#!/bin/bash
# Build A/B on one box: the GPU tests TESTS of the working tree, then bench lines of every side in SIDES
# (ab/<side> copies from tools/ab_build.sh / ab_variant.sh, or "cur") interleaved over ROUNDS rounds for each
# "label|bench args", then a rocprofv3 kernel-stats summary of each side on the first argument set.
#   OUT=r06_c8 SIDES="base cur" TESTS="tests/test_gpu_eg.py tests/test_gpu_eg_fused.py" \
#     tools/gpu_ab.sh "c8|--config c8_decode_eg_1080p" "c8u|--config c8_decode_eg_1080p --kind uniform"
# Any GPU fault / abort / timeout / segfault ends the script: nothing else runs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-gab}
ROOT=$(pwd)
mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 ${PYTEST_TIMEOUT:-400} python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread \
     > $O/pytest.log 2>&1
  rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && { echo "pytest rc=$rc"; exit $rc; }
fi
OUT=${O#gpurun_out/} SIDES="${SIDES:-base cur}" ROUNDS=${ROUNDS:-3} tools/ab_dirs.sh "$@" || exit $?
[ -n "$NO_PROF" ] && exit 0
first=$1; label=${first%%|*}; args=${first#*|}
for side in ${SIDES:-base cur}; do
  dir=.; [ $side != cur ] && dir=ab/$side
  (cd $dir && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $ROOT/$O/prof_$side -o run --output-format csv -- \
     python3 bench.py $args --steps 20 --warmup 5 --no-cpu-baseline --no-ceiling) > $O/prof_$side.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "rocprof $side rc=$rc"; tail -3 $O/prof_$side.log; exit $rc; }
  f=$(find $O/prof_$side -name '*kernel_stats.csv' | head -1); cp "$f" $O/kernel_stats_${label}_$side.csv
  python3 -c "
import csv
for r in csv.DictReader(open('$O/kernel_stats_${label}_$side.csv')):
    if float(r['Calls']) > 10: print('$side', r['Name'][:60], round(float(r['AverageNs'])/1e3,1), 'us')"
done
exit 0
