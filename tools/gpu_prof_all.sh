#!/bin/bash
# Per-config rocprofv3 evidence (run on the GPU box): for each config in CONFIGS
#   1. --kernel-trace --stats              -> gpurun_out/profall/<cfg>/trace/...kernel_stats.csv
#   2. --pmc FETCH_SIZE, 3. --pmc WRITE_SIZE (separate passes, dispatch counters only)
#                                          -> gpurun_out/pmc/<cfg>.csv via tools/pmc_summary.py
# Every pass under its own timeout; the script stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/profall gpurun_out/pmc
for cfg in ${CONFIGS:-c2_encode_1080p c3_decode_1080p c5_encode_1080p_d4 c6_decode_1080p_d4}; do
  d=gpurun_out/profall/$cfg
  mkdir -p $d
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $d/trace -o trace --output-format csv -- \
    python3 bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline --no-ceiling > $d/trace.log 2>&1
  rc=$?; echo "$cfg trace rc=$rc"; grep '^{' $d/trace.log | cut -c1-300; [ $rc -ne 0 ] && { tail -5 $d/trace.log; exit $rc; }
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 240 rocprofv3 --pmc $ctr -d $d/$ctr -o p --output-format csv -- \
      python3 bench.py --config $cfg --steps 4 --warmup 1 --no-cpu-baseline --no-ceiling > $d/$ctr.log 2>&1
    rc=$?; echo "$cfg $ctr rc=$rc"; [ $rc -ne 0 ] && { tail -5 $d/$ctr.log; exit $rc; }
  done
  python3 tools/pmc_summary.py gpurun_out/pmc/$cfg.csv $(find $d/FETCH_SIZE $d/WRITE_SIZE -name "*counter_collection.csv")
done
exit 0
