#!/bin/bash
# PMC HBM-traffic passes (FETCH_SIZE, WRITE_SIZE: separate rocprofv3 --pmc runs, kernel dispatch
# counters only) for each config in CONFIGS; writes gpurun_out/pmc/<config>.csv (copy to profiles/pmc/).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
for cfg in ${CONFIGS:-c2_encode_1080p}; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 240 rocprofv3 --pmc $ctr -d gpurun_out/pmc/$cfg/$ctr -o p --output-format csv -- \
      python3 bench.py --config $cfg --steps 4 --warmup 1 --no-cpu-baseline --no-ceiling > gpurun_out/pmc/$cfg.$ctr.log 2>&1
    rc=$?; echo "$cfg $ctr rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/pmc/$cfg.$ctr.log; exit $rc; }
  done
  python3 tools/pmc_summary.py gpurun_out/pmc/$cfg.csv $(find gpurun_out/pmc/$cfg -name "*counter_collection.csv")
done
