#!/bin/bash
# Runs "name|timeout|command" steps in order on the GPU box; output of each to gpurun_out/$OUT/<name>.log.
# A step that ends in a GPU-fault-like status (abort 134, segfault 139, timeout 124/137, or any
# status > 1 from pytest) stops the script: nothing else runs on the GPU after it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${OUT:-run}
mkdir -p "$OUT"
for step in "$@"; do
  name=${step%%|*}; rest=${step#*|}; tmo=${rest%%|*}; cmd=${rest#*|}
  echo "== $name ($tmo s): $cmd"
  timeout -k 10 "$tmo" bash -c "$cmd" > "$OUT/$name.log" 2>&1
  rc=$?
  tail -4 "$OUT/$name.log"
  echo "== $name rc=$rc"
  case $rc in 0|1) ;; *) echo "stopping after rc=$rc"; exit $rc;; esac
done
exit 0
