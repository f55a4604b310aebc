#!/bin/bash
# Effective shader clock of each config's kernels: GRBM_GUI_ACTIVE (summed over the 8 XCDs) and
# SQ_BUSY_CYCLES in one --pmc pass per config, short bench runs (MI355X_MICROARCH.md: clock ~=
# GRBM_GUI_ACTIVE / 8 / kernel time).  Content-dependent power (DVFS) shows as a lower clock at the same
# instruction count.
#   CONFIGS="c2|--config c2_encode_1080p c2u|--config c2_encode_1080p --kind uniform" tools/gpu_clock.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${OUT:-clock}
mkdir -p $OUT
for v in "$@"; do
  label=${v%%|*}; args=${v#*|}
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_BUSY_CYCLES --kernel-trace \
     -d $OUT/$label -o pmc --output-format csv -- \
     python3 bench.py $args --steps 10 --warmup 3 --no-cpu-baseline --no-ceiling > $OUT/$label.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { tail -5 $OUT/$label.log; echo "stopping: $label rc=$rc"; exit $rc; }
  echo "clock $label collected"
done
