#!/bin/bash
# One GPU session for a round's evidence: the GPU parity suite, then bench lines of the headline
# configs and a rocprofv3 kernel-trace summary of each (the same command as the bench line).
# Any GPU fault / abort / timeout / segfault (124/134/137/139) ends the script: nothing else runs.
#   OUT=gpurun_out/<dir> CONFIGS="c2 c3 ..." SKIP_TESTS=1 tools/gpu_round.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/round}
mkdir -p $OUT
stop() { echo "stopping after rc=$1 ($2)"; exit $1; }
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 ${PYTEST_TIMEOUT:-600} python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
     ${PYTEST_ARGS} > $OUT/pytest_gpu.log 2>&1
  rc=$?; tail -3 $OUT/pytest_gpu.log; echo "pytest rc=$rc"
  [ $rc -ne 0 ] && stop $rc pytest
fi
declare -A CFG=( [c2]="--config c2_encode_1080p" [c2u]="--config c2_encode_1080p --kind uniform"
                 [c3]="--config c3_decode_1080p" [c3u]="--config c3_decode_1080p --kind uniform"
                 [c4]="--config c4_encode_4k" [c5]="--config c5_encode_1080p_d4"
                 [c6]="--config c6_decode_1080p_d4" [c7]="--config c7_encode_eg_1080p"
                 [c8]="--config c8_decode_eg_1080p" [c8u]="--config c8_decode_eg_1080p --kind uniform"
                 [c9]="--config c9_forward_f32_1080p" [c10]="--config c10_inverse_f32_1080p" )
for c in ${CONFIGS:-c2 c2u c3 c4}; do
  extra="--no-cpu-baseline"; [ "$c" = c2 ] && extra=""
  timeout -k 10 240 python bench.py ${CFG[$c]} --steps ${STEPS:-20} --warmup 5 $extra > $OUT/bench_$c.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { tail -5 $OUT/bench_$c.log; stop $rc bench_$c; }
  tail -1 $OUT/bench_$c.log > $OUT/bench_$c.json
  python3 -c "import json; r=json.load(open('$OUT/bench_$c.json')); f=r.get('roofline') or {}; print('$c', round(r['value']/1e9,4), 'G/s ms/step', round(r['ms_per_step'],4), 'frac', f.get('frac'), 'kernel_ms', f.get('kernel_ms'))"
  if [ -z "$NO_PROF" ]; then
    timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/prof_$c -o run --output-format csv -- \
       python3 bench.py ${CFG[$c]} --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline --no-ceiling > $OUT/prof_$c.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { tail -5 $OUT/prof_$c.log; stop $rc prof_$c; }
    f=$(find $OUT/prof_$c -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && cp "$f" $OUT/kernel_stats_$c.csv
    [ -z "$KEEP_TRACE" ] && rm -rf $OUT/prof_$c  # the traces (10+ MiB each; gpurun copies back <= 64 MiB)
  fi
done
exit 0
