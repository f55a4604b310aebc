#!/bin/bash
# Fixed-cost sweep of the encode: bench lines at several batch sizes (kernel_ms and the memory-only
# twin from the same runs), so that T(n) = a + b n separates the per-launch fixed cost a from the
# per-stack rate b.  One line per size into $OUT/sweep.jsonl.
#   OUT=gpurun_out/sweep SIZES="8 16 32 64" CFG="--config c4_encode_4k" KEY=--job-stacks tools/sweep_stacks.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/sweep}
mkdir -p $OUT
CFG=${CFG:-"--config c4_encode_4k"}
KEY=${KEY:---job-stacks}
for n in ${SIZES:-8 16 32 64}; do
  timeout -k 10 180 python bench.py $CFG $KEY $n --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline $EXTRA \
     > $OUT/sweep_$n.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { tail -5 $OUT/sweep_$n.log; echo "stopping: n=$n rc=$rc"; exit $rc; }
  tail -1 $OUT/sweep_$n.log >> $OUT/sweep.jsonl
  python3 -c "import json,sys; r=json.loads(open('$OUT/sweep_$n.log').read().strip().splitlines()[-1]); f=r['roofline']; c=r.get('ceiling') or {}; print('$n', 'step', round(r['ms_per_step'],4), 'kernel', round(f['kernel_ms'],4), 'memonly', c.get('encode_memonly_ms'), 'componly', c.get('encode_computeonly_ms'))"
done
exit 0
