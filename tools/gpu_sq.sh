#!/bin/bash
# SQ counter passes (one --pmc group per pass, kernel dispatch counters only) for the bench in BENCH_ARGS.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/sq${SQ_TAG:+_$SQ_TAG}; mkdir -p $OUT
ARGS=${BENCH_ARGS:-"--steps 6 --warmup 2 --no-cpu-baseline --no-ceiling"}
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU" \
           "SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_LDS" \
           ${SQ_EXTRA:+"$SQ_EXTRA"}; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp -d $OUT/p$i -o p$i --output-format csv -- python3 bench.py $ARGS > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/p$i.log; exit $rc; }
done
python3 tools/pmc_summary.py $OUT/summary.csv $OUT
grep -v "synth" $OUT/summary.csv
