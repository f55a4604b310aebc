#!/bin/bash
# Ramp vs uniform-noise content, one box: for c2 / c2u / c3 / c3u the effective shader
# clock (GRBM_GUI_ACTIVE with a kernel trace, tools/gpu_clock.sh) and the SQ counter groups of
# tools/gpu_sq.sh; summarised by tools/uniform_study.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=${OUT:-uniform}
OUT=$O bash tools/gpu_clock.sh "c2|--config c2_encode_1080p" "c2u|--config c2_encode_1080p --kind uniform" \
   "c3|--config c3_decode_1080p" "c3u|--config c3_decode_1080p --kind uniform" || exit $?
for v in "c2|--config c2_encode_1080p" "c2u|--config c2_encode_1080p --kind uniform" \
         "c3|--config c3_decode_1080p" "c3u|--config c3_decode_1080p --kind uniform"; do
  label=${v%%|*}; args=${v#*|}
  SQ_TAG=${O}_$label BENCH_ARGS="$args --steps 6 --warmup 2 --no-cpu-baseline --no-ceiling --settle-ms 0" \
     SQ_EXTRA="SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" bash tools/gpu_sq.sh > /dev/null || exit $?
  echo "sq $label collected"
done
exit 0
