#!/bin/bash
# Decode evidence on one box: the fp64 issue-rate probe (VALU vs MFMA vs both), then SQ counters of
# decode_kernel (VALU / instruction issue / waits; separate --pmc passes, SQ block only).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${OUT:-decev}
mkdir -p $OUT
timeout -k 10 60 rocprofv3 -L > $OUT/counters.txt 2>&1; echo "list rc=$?"
timeout -k 10 120 tools/bin/f64_rate_probe > $OUT/f64_rate_probe.json 2>&1
rc=$?; echo "probe rc=$rc"; cat $OUT/f64_rate_probe.json; [ $rc -ne 0 ] && exit $rc
CFG=${CFG:-c3_decode_1080p}
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA \
   --kernel-include-regex decode_kernel -d $OUT/sq1 -o sq --output-format csv -- python3 bench.py --config $CFG --steps 4 --warmup 1 --no-cpu-baseline --no-ceiling > $OUT/sq1.log 2>&1
rc=$?; echo "sq1 rc=$rc"; [ $rc -ne 0 ] && { tail -3 $OUT/sq1.log; exit $rc; }
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM \
   --kernel-include-regex decode_kernel -d $OUT/sq2 -o sq --output-format csv -- python3 bench.py --config $CFG --steps 4 --warmup 1 --no-cpu-baseline --no-ceiling > $OUT/sq2.log 2>&1
rc=$?; echo "sq2 rc=$rc"; [ $rc -ne 0 ] && tail -3 $OUT/sq2.log
exit 0
