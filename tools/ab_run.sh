#!/bin/bash
# A/B of two builds on one box: ab/<BASE> (tools/ab_build.sh) against the working tree, alternating
# ROUNDS times (B/N/B/N ...), one bench.py line each; prints value / ms per step / kernel ms / frac.
#   CONFIG=c2_encode_1080p BENCH_ARGS="--kind uniform" ROUNDS=3 tools/ab_run.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${OUT:-ab}
mkdir -p $OUT
ROOT=$(pwd)
for i in $(seq 1 ${ROUNDS:-2}); do
  for side in ${BASE:-base} new; do
    dir=$ROOT; [ $side != new ] && dir=$ROOT/ab/$side
    (cd $dir && timeout -k 10 200 python bench.py --config ${CONFIG:-c2_encode_1080p} --steps ${STEPS:-20} --warmup 5 \
       --no-cpu-baseline ${BENCH_ARGS}) > $OUT/${side}_$i.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { tail -5 $OUT/${side}_$i.log; echo "stopping: $side rc=$rc"; exit $rc; }
    python3 -c "import json; r=json.loads(open('$OUT/${side}_$i.log').read().strip().splitlines()[-1]); f=r['roofline']; c=r.get('ceiling') or {}; print('$side', round(r['value']/1e9,4), 'G/s ms/step', round(r['ms_per_step'],4), 'kernel_ms', round(f['kernel_ms'],4), 'frac', round(f['frac'],4), 'memonly_ms', c.get('encode_memonly_ms') or c.get('decode_memonly_ms'))"
  done
done
