#!/bin/bash
# A/B of bench.py argument sets on one box, interleaved over ROUNDS rounds (box drift hits every
# variant alike).  Each argument is "label|bench args"; one summary line per run:
#   ROUNDS=2 tools/ab_args.sh "s0|--config c4_encode_4k --job-stacks 8" "s4|... --opt enc_stagger=4"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${OUT:-ab}
mkdir -p $OUT
for i in $(seq 1 ${ROUNDS:-2}); do
  for v in "$@"; do
    label=${v%%|*}; args=${v#*|}
    timeout -k 10 180 python bench.py $args --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline --no-ceiling \
       > $OUT/${label}_$i.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { tail -5 $OUT/${label}_$i.log; echo "stopping: $label rc=$rc"; exit $rc; }
    tail -1 $OUT/${label}_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$label', $i, 'ms/step', round(d['ms_per_step'],4), 'kernel', round(r['kernel_ms'],4), 'frac', round(r['frac'],4), 'aux', round(r.get('aux_ms') or 0,4), 'rechecked', d.get('rechecked_units_last_step'))"
  done
done
exit 0
