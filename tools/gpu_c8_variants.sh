#!/bin/bash
# c8 A/B of several builds on one box: the GPU Exp-Golomb / codec tests of the working tree, then c8
# bench lines of each side (ab/<side> or "cur") interleaved over ROUNDS rounds (ramp and uniform), then
# per side a rocprofv3 kernel trace and the SQ counter passes of the parse kernels.
#   SIDES="base lin cur" OUT=r05_c8 ROUNDS=3 tools/gpu_c8_variants.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
ROOT=$(pwd)
O=$ROOT/gpurun_out/${OUT:-c8var}
mkdir -p $O
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 500 python -u -m pytest ${TESTS:-tests/test_gpu_eg.py tests/test_gpu_eg_fused.py tests/test_gpu_codec.py} \
     -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
  rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && { echo "pytest rc=$rc"; exit $rc; }
fi
CFG=${CONFIG:-c8_decode_eg_1080p}
for i in $(seq 1 ${ROUNDS:-3}); do
  for kind in ${KINDS:-ramp uniform}; do
    for side in ${SIDES:-base cur}; do
      dir=$ROOT; [ $side != cur ] && dir=$ROOT/ab/$side
      (cd $dir && timeout -k 10 200 python bench.py --config $CFG --kind $kind --steps 20 --warmup 5 \
         --no-cpu-baseline --no-ceiling) > $O/${side}_${kind}_$i.log 2>&1
      rc=$?; [ $rc -ne 0 ] && { tail -5 $O/${side}_${kind}_$i.log; echo "stopping: $side rc=$rc"; exit $rc; }
      python3 -c "import json; r=json.loads(open('$O/${side}_${kind}_$i.log').read().strip().splitlines()[-1]); f=r['roofline']; print('$side $kind $i', round(r['value']/1e9,4), 'G/s ms/step', round(r['ms_per_step'],4), 'kernel_ms', round(f['kernel_ms'],4))"
    done
  done
done
[ -n "$NO_PROF" ] && exit 0
for side in ${SIDES:-base cur}; do
  dir=$ROOT; [ $side != cur ] && dir=$ROOT/ab/$side
  (cd $dir && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_$side -o run --output-format csv -- \
     python3 bench.py --config $CFG --steps 20 --warmup 5 --no-cpu-baseline --no-ceiling) \
     > $O/prof_$side.log 2>&1 || { echo "rocprof $side failed"; tail -3 $O/prof_$side.log; exit 1; }
  f=$(find $O/prof_$side -name '*kernel_stats.csv' | head -1); cp "$f" $O/kernel_stats_$side.csv
  python3 -c "
import csv
for r in csv.DictReader(open('$O/kernel_stats_$side.csv')):
    if 'eg_' in r['Name'] or 'decode_eg' in r['Name']: print('$side', r['Name'][:50], round(float(r['AverageNs'])/1e3,1), 'us')"
done
[ -n "$NO_SQ" ] && exit 0
for side in ${SQ_SIDES:-base cur}; do
  dir=$ROOT; [ $side != cur ] && dir=$ROOT/ab/$side
  j=0
  for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
             "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU" \
             "SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_LDS" \
             "FETCH_SIZE" "WRITE_SIZE"; do
    j=$((j+1))
    (cd $dir && timeout -s KILL 120 rocprofv3 --pmc $grp -d $O/sq_$side/p$j -o p$j --output-format csv -- \
       python3 bench.py --config $CFG --steps 4 --warmup 1 --no-cpu-baseline --no-ceiling) > $O/sq_${side}_p$j.log 2>&1
    rc=$?; echo "sq $side pass $j rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/sq_${side}_p$j.log; exit $rc; }
  done
  python3 tools/pmc_summary.py $O/sq_summary_$side.csv $O/sq_$side > /dev/null 2>&1
  grep -E "eg_|decode_eg" $O/sq_summary_$side.csv | cut -c1-200
done
exit 0
