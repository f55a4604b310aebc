cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for cfg in c2_encode_1080p c3_decode_1080p c4_encode_4k c5_encode_1080p_d4 c6_decode_1080p_d4 c7_encode_eg_1080p c8_decode_eg_1080p c9_forward_f32_1080p c10_inverse_f32_1080p; do
  extra=""; [ "$cfg" != "c2_encode_1080p" ] && extra="--no-cpu-baseline"
  timeout -k 10 300 python bench.py --config $cfg --steps 20 --warmup 5 $extra > gpurun_out/bench_$cfg.log 2>&1
  rc=$?; echo "bench $cfg rc=$rc"; grep '^{' gpurun_out/bench_$cfg.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['ms_per_step'], r['frac'], r['kernel_ms'])"; [ $rc -ne 0 ] && exit $rc
done
CONFIGS="c2_encode_1080p c7_encode_eg_1080p" bash tools/gpu_prof_all.sh
