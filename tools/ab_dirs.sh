#!/bin/bash
# A/B of builds on one box: ab/<side> copies (git archive + make) against the working
# tree ("cur"), interleaved over ROUNDS rounds, for each argument set "label|bench args".
#   SIDES="base cur" ROUNDS=2 tools/ab_dirs.sh "c2|" "c2u|--kind uniform"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/${OUT:-abd}
mkdir -p $OUT
for i in $(seq 1 ${ROUNDS:-2}); do
  for v in "$@"; do
    label=${v%%|*}; args=${v#*|}
    for side in ${SIDES:-base cur}; do
      dir=.; [ $side != cur ] && dir=ab/$side
      (cd $dir && timeout -k 10 180 python bench.py $args --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline --no-ceiling) \
         > $OUT/${label}_${side}_$i.log 2>&1
      rc=$?; [ $rc -ne 0 ] && { tail -5 $OUT/${label}_${side}_$i.log; echo "stopping: $label $side rc=$rc"; exit $rc; }
      tail -1 $OUT/${label}_${side}_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$label', '$side', $i, 'ms/step', round(d['ms_per_step'],4), 'kernel', round(r['kernel_ms'],4), 'frac', round(r['frac'],4), 'rechecked', d.get('rechecked_units_last_step'))"
    done
  done
done
exit 0
