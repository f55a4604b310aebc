#!/bin/bash
# rocprofv3 passes for the headline bench (run on the GPU box):
#   1. kernel trace + stats (per-kernel average durations)
#   2. --pmc FETCH_SIZE   (separate pass: TCC slot budget; gfx950: FETCH_SIZE reads 1/2 of a wide
#                          coalesced stream, see MI355X_MICROARCH.md §HBM)
#   3. --pmc WRITE_SIZE
# Each pass under its own timeout; stops at the first crash/timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof${PROF_TAG:+_$PROF_TAG}
mkdir -p $OUT
ARGS=${BENCH_ARGS:-"--steps 10 --warmup 3 --no-cpu-baseline"}
run() {
  local name=$1; shift
  timeout -k 10 300 rocprofv3 "$@" -d $OUT/$name -o $name --output-format csv -- python3 bench.py $ARGS > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -2 $OUT/$name.log
  case $rc in 0) ;; *) exit $rc;; esac
}
run trace --kernel-trace --stats
[ -n "$TRACE_ONLY" ] && exit 0
run fetch --pmc FETCH_SIZE
run write --pmc WRITE_SIZE
find $OUT -name "*.csv" | head -20
