#!/bin/bash
# Occupancy sweep (blocks per CU via dynamic LDS padding) for the encode and decode kernels.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/occ
for pad in ${PADS:-0 6 20 44}; do
  for cfg in ${CONFIGS:-c2_encode_1080p c3_decode_1080p}; do
    DCT3D_ENC_LDS_PAD_KB=$pad DCT3D_DEC_LDS_PAD_KB=$pad timeout -k 10 200 python bench.py --config $cfg --steps 20 --warmup 5 \
      --no-cpu-baseline --no-ceiling > gpurun_out/occ/${cfg}_$pad.log 2>&1 || exit $?
    python3 -c "import json; r=json.loads(open('gpurun_out/occ/${cfg}_$pad.log').read().strip().splitlines()[-1]); print('$cfg pad=${pad}KiB', round(r['value']/1e9,4), 'Gcubes/s kernel_ms', round(r['roofline']['kernel_ms'],4), 'frac', round(r['roofline']['frac'],4))"
  done
done
