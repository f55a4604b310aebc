#!/bin/bash
# Bench with the bandwidth ceiling probe, then one SQ-counter pass on the encode kernel.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/probe
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/probe/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/probe/bench.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['value'], r['roofline']['kernel_ms'], r['roofline']['frac'], r['ceiling'])"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES \
   --kernel-include-regex encode_kernel -d gpurun_out/probe/sq -o sq --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-ceiling > gpurun_out/probe/sq.log 2>&1
echo "sq rc=$?"; tail -3 gpurun_out/probe/sq.log
exit 0
