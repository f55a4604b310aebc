#!/bin/bash
# A/B of two builds on one box: ab/<BASE> (tools/ab_build.sh) against the working tree, config CONFIG
# (default c7_encode_eg_1080p).  The GPU tests TESTS of the working tree, then ROUNDS interleaved bench
# lines per side (ramp, and uniform content with UNIFORM=1), then a rocprofv3 kernel trace of each side
# for the per-kernel split.
#   BASE=base OUT=r04_c7ab ROUNDS=3 UNIFORM=1 tools/gpu_build_ab.sh
#   CONFIG=c8_decode_eg_1080p TESTS="tests/test_gpu_eg.py tests/test_gpu_eg_fused.py" tools/gpu_build_ab.sh
# NEW=<name>: the "new" side from ab/<name> instead of the working tree (the tests still run here).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-buildab}; B=${BASE:-base}; CFG=${CONFIG:-c7_encode_eg_1080p}; TAG=${CFG%%_*}
mkdir -p $O
ROOT=$(pwd)
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_gpu_eg_fused.py tests/test_gpu_codec.py} -m gpu -x -q --timeout 120 \
     --timeout-method thread > $O/pytest.log 2>&1
  rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && { echo "pytest rc=$rc"; exit $rc; }
fi
kinds="ramp"; [ -n "$UNIFORM" ] && kinds="ramp uniform"
for i in $(seq 1 ${ROUNDS:-3}); do
  for kind in $kinds; do
    for side in $B new; do
      dir=$ROOT; [ $side != new ] && dir=$ROOT/ab/$side; [ $side = new ] && [ -n "$NEW" ] && dir=$ROOT/ab/$NEW
      (cd $dir && timeout -k 10 200 python bench.py --config $CFG --kind $kind --steps 20 --warmup 5 \
         --no-cpu-baseline --no-ceiling) > $O/${side}_${kind}_$i.log 2>&1
      rc=$?; [ $rc -ne 0 ] && { tail -5 $O/${side}_${kind}_$i.log; echo "stopping: $side rc=$rc"; exit $rc; }
      python3 -c "import json; r=json.loads(open('$O/${side}_${kind}_$i.log').read().strip().splitlines()[-1]); f=r['roofline']; print('$side $kind', round(r['value']/1e9,4), 'G/s ms/step', round(r['ms_per_step'],4), 'kernel_ms', round(f['kernel_ms'],4))"
    done
  done
done
[ -n "$NO_PROF" ] && exit 0
for side in $B new; do
  dir=$ROOT; [ $side != new ] && dir=$ROOT/ab/$side; [ $side = new ] && [ -n "$NEW" ] && dir=$ROOT/ab/$NEW
  (cd $dir && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $ROOT/$O/prof_$side -o run --output-format csv -- \
     python3 bench.py --config $CFG --steps 20 --warmup 5 --no-cpu-baseline --no-ceiling) \
     > $O/prof_$side.log 2>&1 || { echo "rocprof $side failed"; tail -3 $O/prof_$side.log; exit 1; }
  f=$(find $O/prof_$side -name '*kernel_stats.csv' | head -1); cp "$f" $O/kernel_stats_${TAG}_$side.csv
  python3 -c "
import csv
for r in csv.DictReader(open('$O/kernel_stats_${TAG}_$side.csv')):
    print('$side', r['Name'][:60], round(float(r['AverageNs'])/1e3,1), 'us')"
done
exit 0
