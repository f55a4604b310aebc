#!/bin/bash
# HBM traffic of each config's kernels: FETCH_SIZE and WRITE_SIZE in separate rocprofv3 --pmc passes
# (TCC slots: 3 + 2 > 4), short bench runs, then the per-kernel summary profiles/pmc/<config>.csv that
# bench.py reads for roofline.traffic (FETCH_SIZE x2 on gfx950: MI355X_MICROARCH.md, HBM section).
#   CONFIGS="c2_encode_1080p c3_decode_1080p" tools/gpu_pmc.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${OUT:-pmc}
mkdir -p $OUT profiles/pmc
for cfg in ${CONFIGS:-c2_encode_1080p c3_decode_1080p}; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $ctr -d $OUT/${cfg}_$ctr -o pmc --output-format csv -- \
       python3 bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline --no-ceiling > $OUT/${cfg}_$ctr.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { tail -5 $OUT/${cfg}_$ctr.log; echo "stopping: $cfg $ctr rc=$rc"; exit $rc; }
  done
  echo "pmc $cfg collected"
done
# then, here: python3 tools/pmc_summary.py profiles/pmc/<cfg>.csv gpurun_out/pmc/<cfg>_FETCH_SIZE gpurun_out/pmc/<cfg>_WRITE_SIZE
