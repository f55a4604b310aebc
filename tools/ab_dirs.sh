#!/bin/bash
# A/B of whole builds on one box: for each run in RUNS ("dir" = a tree under ab/ or "." for the
# working tree), one bench of CONFIG (ARGS extra); prints dir / value / kernel ms per run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
i=0
for d in ${RUNS:-. ab/base . ab/base}; do
  i=$((i+1))
  (cd $d && timeout -k 10 200 python bench.py --config ${CONFIG:-c2_encode_1080p} --steps 20 --warmup 5 --no-cpu-baseline ${ARGS}) > gpurun_out/ab/dirs_$i.log 2>&1
  rc=$?; case $rc in 0) ;; *) echo "$d bench rc=$rc"; tail -3 gpurun_out/ab/dirs_$i.log; exit $rc;; esac
  python3 -c "import json; r=json.loads(open('gpurun_out/ab/dirs_$i.log').read().strip().splitlines()[-1]); c=r.get('ceiling') or {}; print('$d', round(r['value']/1e9,4),'Gcubes/s ms/step', round(r['ms_per_step'],4), 'kernel_ms', round(r['roofline']['kernel_ms'],4), 'frac', round(r['roofline']['frac'],4), 'memonly', round(c.get('encode_memonly_ms',0),4))"
done
