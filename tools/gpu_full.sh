#!/bin/bash
# Full GPU session: all -m gpu tests, smoke(), then the bench for every BASELINE config.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
stop() { case $1 in 0|1) ;; *) echo "stopping after rc=$1"; exit $1;; esac; }
timeout -k 10 900 python -m pytest tests -m gpu -q ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_gpu.log; echo "pytest rc=$rc"; stop $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -2 gpurun_out/smoke.log; echo "smoke rc=$rc"; stop $rc
for cfg in ${CONFIGS:-c2_encode_1080p c3_decode_1080p c5_encode_1080p_d4 c4_encode_4k}; do
  extra=""; [ "$cfg" != "c2_encode_1080p" ] && extra="--no-cpu-baseline"
  timeout -k 10 300 python bench.py --config $cfg --steps 20 --warmup 5 $extra > gpurun_out/bench_$cfg.log 2>&1
  rc=$?; echo "bench $cfg rc=$rc"; tail -1 gpurun_out/bench_$cfg.log | cut -c1-400; [ $rc -ne 0 ] && exit $rc
done
exit 0
