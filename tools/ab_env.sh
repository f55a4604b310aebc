#!/bin/bash
# A/B of an environment knob on one box: for each value in VALUES, the parity subset TESTS (pytest -k)
# then one bench run of CONFIG; prints value / kernel_ms per run.  VAR=name of the knob.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
i=0
for v in ${VALUES:-1 0 1 0}; do
  i=$((i+1))
  if [ -n "$TESTS" ]; then
    env $VAR=$v timeout -k 10 300 python -m pytest tests -m gpu -x -q -k "$TESTS" > gpurun_out/ab/pytest_$i.log 2>&1
    rc=$?; echo "$VAR=$v pytest rc=$rc $(tail -1 gpurun_out/ab/pytest_$i.log)"
    case $rc in 0) ;; *) exit $rc;; esac
  fi
  env $VAR=$v timeout -k 10 200 python bench.py --config ${CONFIG:-c2_encode_1080p} --steps 20 --warmup 5 --no-cpu-baseline --no-ceiling > gpurun_out/ab/bench_$i.log 2>&1
  rc=$?; case $rc in 0) ;; *) echo "bench rc=$rc"; exit $rc;; esac
  python3 -c "import json; r=json.loads(open('gpurun_out/ab/bench_$i.log').read().strip().splitlines()[-1]); print('$VAR=$v', round(r['value']/1e9,4),'Gcubes/s ms/step', round(r['ms_per_step'],4), 'kernel_ms', round(r['roofline']['kernel_ms'],4), 'frac', round(r['roofline']['frac'],4))"
done
