#!/bin/bash
# A/B of the c7 bench between ab/<BASE> and the working tree, alternating, one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
BASE=${BASE:-v1}; CFG=${CFG:-c7_encode_eg_1080p}
for i in 1 2; do
  for side in $BASE cur; do
    dir=.; [ $side != cur ] && dir=ab/$side
    (cd $dir && timeout -k 10 200 python bench.py --config $CFG --steps 20 --warmup 5 --no-cpu-baseline --no-ceiling $BENCH_ARGS) > gpurun_out/ab/${side}_$i.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "$side rc=$rc"; tail -5 gpurun_out/ab/${side}_$i.log; exit $rc; }
    grep '^{' gpurun_out/ab/${side}_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$side', round(d['value']/1e9,4), 'ms/step', round(d['ms_per_step'],3), 'kernel', round(r['kernel_ms'],3), 'rest', round(r.get('aux_ms', r.get('fixup_ms', 0.0)),3))"
  done
done
