#!/bin/bash
# One GPU session: parity tests, then (only if no crash) a short bench.  Exit codes 124/134/137/139
# stop the script (GPU fault / abort / timeout / segfault): nothing else runs on the GPU after them.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -m pytest tests -m gpu -x -q ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -25 gpurun_out/pytest_gpu.log
echo "pytest rc=$rc"
case $rc in 0|1) ;; *) echo "stopping after rc=$rc"; exit $rc;; esac
timeout -k 10 ${BENCH_TIMEOUT:-300} python bench.py --steps ${STEPS:-10} --warmup 3 ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
brc=$?
tail -5 gpurun_out/bench.log
echo "bench rc=$brc"
exit $brc
