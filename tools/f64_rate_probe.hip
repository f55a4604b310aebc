// f64_rate_probe.hip -- standalone fp64 issue-rate probe (tool, not part of the product library).
// The north_star asks for MFMA only if it wins.  The decode runs fp64 (its certificate needs it), so
// the question is whether the 8-point inverse passes would run faster on v_mfma_f64_16x16x4_f64 than
// as VALU butterflies, or beside them.  This measures, on the device:
//   1. VALU  : v_fma_f64 (8 independent chains per lane), FLOP/s over the chip;
//   2. MFMA  : v_mfma_f64_16x16x4_f64 (4 independent accumulators per wave), FLOP/s;
//   3. MIXED : half of each block's waves on (1), half on (2) -- do the two pipes add up?
// and derives the per-line cost of an 8-point inverse DCT both ways (butterfly: 36 fp64 ops per line
// on the VALU; MFMA: a dense 8x8 product, 64 MAC per line, with the 16x16x4 shape filled at most
// half by one 8-point basis).
//   build: hipcc --offload-arch=gfx950 -O3 -o tools/bin/f64_rate_probe tools/f64_rate_probe.hip
//   run:   tools/bin/f64_rate_probe
#include <hip/hip_runtime.h>

#include <cstdio>

typedef double f64x4 __attribute__((ext_vector_type(4)));

constexpr int kIters = 4096;

__device__ __forceinline__ void valu_body(double* sink, int lane) {
    double a[8];
#pragma unroll
    for (int i = 0; i < 8; i++) a[i] = 1.0 + 1e-9 * (lane + i);
    const double b = 0.999999, c = 1e-7;
    for (int it = 0; it < kIters; it++) {
#pragma unroll
        for (int i = 0; i < 8; i++) a[i] = __fma_rn(a[i], b, c);
    }
    double s = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) s += a[i];
    if (s == 12345.0) sink[lane] = s;  // never true: keeps the work
}

__device__ __forceinline__ void mfma_body(double* sink, int lane) {
    f64x4 acc[4];
#pragma unroll
    for (int i = 0; i < 4; i++) acc[i] = f64x4{0, 0, 0, 0};
    const double a = 1.0 + 1e-9 * lane, b = 0.5;
    for (int it = 0; it < kIters / 4; it++) {
#pragma unroll
        for (int i = 0; i < 4; i++) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
    }
    double s = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    if (s == 12345.0) sink[lane] = s;
}

template <int MODE>  // 0 VALU, 1 MFMA, 2 mixed (even waves VALU, odd waves MFMA)
__global__ __launch_bounds__(256) void probe(double* sink) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (MODE == 0 || (MODE == 2 && (wave & 1) == 0)) valu_body(sink, lane);
    else mfma_body(sink, lane);
}

template <int MODE>
static float run(double* sink, int blocks) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(probe<MODE>, dim3(blocks), dim3(256), 0, 0, sink);  // warm-up
    hipEventRecord(e0);
    hipLaunchKernelGGL(probe<MODE>, dim3(blocks), dim3(256), 0, 0, sink);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    return ms;
}

int main() {
    int dev = 0, cus = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    double* sink;
    if (hipMalloc(&sink, 64 * sizeof(double)) != hipSuccess) return 1;
    const int blocks = cus * 8;  // 32 waves per CU
    const double waves = blocks * 4.0;
    // FLOP per wave: VALU 8 chains x kIters fma x 64 lanes x 2; MFMA kIters MFMAs x 16*16*4*2
    const double fv = 8.0 * kIters * 64 * 2, fm = (double)kIters * 16 * 16 * 4 * 2;
    const float tv = run<0>(sink, blocks), tm = run<1>(sink, blocks), tx = run<2>(sink, blocks);
    const double valu_tf = waves * fv / (tv * 1e-3) / 1e12, mfma_tf = waves * fm / (tm * 1e-3) / 1e12;
    const double mixed_tf = (waves / 2 * fv + waves / 2 * fm) / (tx * 1e-3) / 1e12;
    printf("{\"cus\": %d, \"valu_f64_TFLOPs\": %.2f, \"mfma_f64_TFLOPs\": %.2f, \"mixed_TFLOPs\": %.2f, "
           "\"mixed_vs_sum\": %.3f, \"valu_ms\": %.3f, \"mfma_ms\": %.3f, \"mixed_ms\": %.3f,",
           cus, valu_tf, mfma_tf, mixed_tf, mixed_tf / (valu_tf + mfma_tf), tv, tm, tx);
    // 8-point inverse line: butterfly 36 fp64 ops (idct8: 20 add + 16 fma/mul) on the VALU; MFMA:
    // 64 MAC dense, 16x16x4 at most half filled by an 8x8 basis -> 128 MAC slots = 256 FLOP-slots
    const double valu_lines = valu_tf * 1e12 / 2 / 36.0, mfma_lines = mfma_tf * 1e12 / 256.0;
    printf(" \"idct8_lines_per_s_valu\": %.3e, \"idct8_lines_per_s_mfma\": %.3e, \"mfma_over_valu\": %.3f}\n",
           valu_lines, mfma_lines, mfma_lines / valu_lines);
    hipFree(sink);
    return 0;
}
