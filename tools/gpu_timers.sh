#!/bin/bash
# The headline's timers against its kernel trace, and config 1's CPU line:
#   OUT=r04_timers tools/gpu_timers.sh      -> gpurun_out/$OUT/{timed_trace_c2.json, bench_c1.json, ...}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-timers}
mkdir -p $O
for c in ${CONFIGS:-c2}; do
  case $c in
    c2) args="--config c2_encode_1080p"; k=encode16_kernel;;
    c3) args="--config c3_decode_1080p"; k=decode_kernel;;
    c5) args="--config c5_encode_1080p_d4"; k=encode_kernel;;
  esac
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_$c -o run --output-format csv -- \
     python3 bench.py $args --steps 20 --warmup 5 --no-cpu-baseline --no-ceiling > $O/prof_$c.log 2>&1 \
     || { echo "rocprof $c failed"; tail -3 $O/prof_$c.log; exit 1; }
  f=$(find $O/prof_$c -name '*kernel_trace.csv' | head -1)
  python3 tools/timed_trace.py "$f" $O/prof_$c.log $k --out $O/timed_trace_$c.json | grep -v '^  *[0-9]' | head -30
  cp $(find $O/prof_$c -name '*kernel_stats.csv' | head -1) $O/kernel_stats_$c.csv
done
if [ -z "$NO_C1" ]; then
  timeout -k 10 300 python3 bench.py --config c1_java_cpu_64x64 --steps ${C1_STEPS:-400} --warmup 5 > $O/bench_c1.log 2>&1 \
     || { echo "c1 failed"; tail -3 $O/bench_c1.log; exit 1; }
  tail -1 $O/bench_c1.log > $O/bench_c1.json
  python3 -c "import json; d=json.load(open('$O/bench_c1.json')); print('c1', round(d['value']), d['unit'], 'threads', d['cpu_baseline']['cores'], 'ms/step', round(d['ms_per_step'],3))"
fi
exit 0
