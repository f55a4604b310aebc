// dct3d_kernels_f.hip -- fp64 DCT output from the raster (fp64 internal arithmetic):
//   (the drop-in (A) float kernel, cube_f32_kernel, shares the decode's geometry and lives in
//   dct3d_kernels.hip)
//   * fwd64_raster_kernel<D>: fp64 DCT coefficients straight from the u8 raster (the Java dctCoeff
//     values, DCT.java:41-59) for the float-DCT parity output of dct3d_encode_stacks.
// Same wave decomposition as dct3d_kernels.hip (8 cubes per wave, 8 lanes per cube, one
// wave-private LDS transpose done in four 16-byte quarter rounds because the values are fp64).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "dct_butterfly.h"
#include "dct3d_kernels.h"

namespace dct3d {

namespace {
constexpr int kWavesPerBlockF = 4;
constexpr int kSlotF = 144;
constexpr int kWaveLdsF = kSlotF * 64;

__device__ __forceinline__ void wave_sync_f() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
}  // namespace

// Row layout (c, y = j) -> face layout (c, j): writer holds a[kz][kx], reader gets b[y][kx'].
template <int D, int NB>
__device__ __forceinline__ void row_to_face(const double (&a)[D][8], double (&b)[8][NB], int c, int j, char* wl) {
#pragma unroll
    for (int qr = 0; qr < 4; qr++) {
#pragma unroll
        for (int kz = 0; kz < D; kz++)
            *(double2*)(wl + (c * D + kz) * kSlotF + j * 16) = make_double2(a[kz][2 * qr], a[kz][2 * qr + 1]);
        wave_sync_f();
        const bool reader = (D == 8) || ((j & 1) == (qr >> 1));
        if (reader) {
            const int kz = (D == 8) ? j : (j >> 1);
            const int xl = (D == 8) ? 2 * qr : 2 * (qr & 1);
#pragma unroll
            for (int y = 0; y < 8; y++) {
                const double2 t = *(const double2*)(wl + (c * D + kz) * kSlotF + y * 16);
                b[y][xl] = t.x;
                b[y][xl + 1] = t.y;
            }
        }
        wave_sync_f();
    }
}

template <int D>
__global__ __launch_bounds__(256) void fwd64_raster_kernel(Fwd64Params P) {
    constexpr int CS = 64 * D;
    constexpr int NB = (D == 8) ? 8 : 4;
    __shared__ __attribute__((aligned(16))) char lds[kWavesPerBlockF * kWaveLdsF];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int c = lane >> 3, j = lane & 7;
    char* wl = lds + wave * kWaveLdsF;
    const uint32_t g = (blockIdx.x * kWavesPerBlockF + wave) * 8 + c;
    const bool valid = g < P.n_cubes;
    double a[D][8];
    if (valid) {
        const uint32_t s = g / P.cubes_per_stack;
        const uint32_t r = g - s * P.cubes_per_stack;
        const uint32_t by = r / P.nbx, bx = r - by * P.nbx;
        const uint8_t* src = P.raster + (size_t)s * P.stack_stride + (size_t)(by * 8 + j) * P.width + bx * 8;
#pragma unroll
        for (int z = 0; z < D; z++) {
            const uint2 v = *(const uint2*)(src + (size_t)z * P.plane);
#pragma unroll
            for (int e = 0; e < 4; e++) {
                a[z][e] = (double)((v.x >> (8 * e)) & 0xFF);
                a[z][e + 4] = (double)((v.y >> (8 * e)) & 0xFF);
            }
        }
    } else {
#pragma unroll
        for (int z = 0; z < D; z++)
#pragma unroll
            for (int x = 0; x < 8; x++) a[z][x] = 0.0;
    }
#pragma unroll
    for (int z = 0; z < D; z++) fdct8<false, false>(a[z], 0.0);
#pragma unroll
    for (int x = 0; x < 8; x++) {
        double col[D];
#pragma unroll
        for (int z = 0; z < D; z++) col[z] = a[z][x];
        fdctN<D, false, false>(col, 0.0);
#pragma unroll
        for (int z = 0; z < D; z++) a[z][x] = col[z];
    }
    double b[8][NB];
    row_to_face<D, NB>(a, b, c, j, wl);
#pragma unroll
    for (int x = 0; x < NB; x++) {
        double col[8];
#pragma unroll
        for (int y = 0; y < 8; y++) col[y] = b[y][x];
        fdct8<false, false>(col, 0.0);
#pragma unroll
        for (int y = 0; y < 8; y++) b[y][x] = col[y];
    }
    if (valid) {
        const int kz = (D == 8) ? j : (j >> 1);
        const int x0 = (D == 8) ? 0 : (j & 1) * 4;
        double* o = P.out + (size_t)g * CS + kz * 64 + x0;
#pragma unroll
        for (int y = 0; y < 8; y++)
#pragma unroll
            for (int x = 0; x < NB; x += 2) *(double2*)(o + y * 8 + x) = make_double2(b[y][x], b[y][x + 1]);
    }
}

int launch_fwd64_raster(int D, const Fwd64Params& P, hipStream_t st) {
    const uint32_t blocks = (P.n_cubes + 31) / 32;
    if (!blocks) return 0;
    if (D == 8) hipLaunchKernelGGL(fwd64_raster_kernel<8>, dim3(blocks), dim3(256), 0, st, P);
    else hipLaunchKernelGGL(fwd64_raster_kernel<4>, dim3(blocks), dim3(256), 0, st, P);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace dct3d
