#!/bin/bash
# Kernel variant sweep: parity subset + bench per variant, one box.
#   VAR_ENV=DCT3D_ENC_VARIANT (default) or DCT3D_DEC_VARIANT; TESTS = pytest -k expression.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/sweep
VE=${VAR_ENV:-DCT3D_ENC_VARIANT}
K=${TESTS:-encode_64x64 or ragged or encode_1080p_stack or overflow or depth4}
i=0
for v in ${VARIANTS:-0 1 2}; do
  i=$((i+1))
  env $VE=$v timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "$K" > gpurun_out/sweep/pytest_v$v.log 2>&1
  rc=$?; echo "variant $v pytest rc=$rc $(tail -1 gpurun_out/sweep/pytest_v$v.log)"
  case $rc in 0|1) ;; *) exit $rc;; esac
  env $VE=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/sweep/bench_${i}_v$v.log 2>&1
  rc=$?; case $rc in 0) ;; *) echo "bench rc=$rc"; exit $rc;; esac
  python3 -c "import json,sys; r=json.loads(open('gpurun_out/sweep/bench_${i}_v$v.log').read().strip().splitlines()[-1]); print('variant $v', round(r['value']/1e9,4),'Gcubes/s', 'kernel_ms', round(r['roofline']['kernel_ms'],4), 'frac', round(r['roofline']['frac'],4), 'fixup_ms', round(r['roofline']['fixup_ms'],4))"
done
