// dct3d_dev.h -- device helpers shared by the product kernels (dct3d_kernels.hip) and the
// diagnostic kernels (dct3d_diag.hip): launch geometry, wave-level LDS ordering, Java rounding,
// register pins, FastDiv.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>

#include "dct_butterfly.h"
#include "dct3d_eg_bits.h"
#include "dct3d_kernels.h"

namespace dct3d {

constexpr int kWave = 64;
constexpr int kCubesPerWave = 8;
constexpr int kWavesPerBlock = 4;
constexpr int kBlock = kWave * kWavesPerBlock;
constexpr int kSlot = 144;                 // transpose slot: 8 rows x 16 B + 16 B pad (bank spread)
constexpr int kWaveLds = kSlot * 64;       // 9216 B per wave
constexpr int kFace = 272;                 // staging face: 256 B + 16 B pad
static_assert(4 * 8 * kFace <= kWaveLds, "staging round must fit the wave region");
// per-wave LDS of the encode kernels: 8x8x4 moves its transpose and staging in two half rounds
// (4.5 KiB), so that LDS does not cap it at 16 waves per CU (it needs 96 VGPRs: 5 waves per SIMD)
template <int D> constexpr int enc_wave_lds() { return D == 8 ? kWaveLds : kWaveLds / 2; }

// XCD-aware tile order: the dispatcher deals blocks to the 8 XCDs round-robin, so consecutive tiles
// land on 8 different XCDs (each with its own L2).  G = 0: block b takes tile (b % 8) * (nb / 8) + b / 8,
// each XCD walks a contiguous eighth of the data; G > 0: each XCD walks runs of G consecutive tiles
// (tiles 8G apart between its runs).  Measured per kernel (profiles/r02/variant_sweep.txt).
template <uint32_t G = 0>
__device__ __forceinline__ uint32_t xcd_tile() {
    if constexpr (G == 0) {
        const uint32_t nb8 = gridDim.x / 8u;
        return blockIdx.x < nb8 * 8u ? (blockIdx.x & 7u) * nb8 + (blockIdx.x >> 3) : blockIdx.x;
    } else {
        const uint32_t full = gridDim.x / (8u * G) * (8u * G);
        if (blockIdx.x >= full) return blockIdx.x;
        const uint32_t r = blockIdx.x >> 3;
        return (r / G) * (8u * G) + (blockIdx.x & 7u) * G + (r % G);
    }
}
static_assert(4 * 4 * kFace <= kWaveLds / 2, "8x8x4 staging round must fit the half region");

// Wave-level ordering of LDS traffic between lanes of ONE wave: a compiler fence (LDS instructions
// of a wave are executed in order, so no s_waitcnt is needed for visibility within the wave).
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Java Math.round(double) (round half up, exact)
__device__ __forceinline__ int java_round_dev(double a) {
    double f = floor(a);
    return (int)f + ((a - f) >= 0.5 ? 1 : 0);
}

// Register "pins": an empty volatile asm that redefines the values passed to it.  Volatile asms keep
// program order, so pinning a butterfly's inputs before it and its outputs after it serialises the
// butterflies of a pass (the compiler otherwise interleaves all of them and multiplies the live
// temporaries, which costs occupancy).
template <class T, int N>
__device__ __forceinline__ void pin2(T (&x)[N], T (&y)[N]) {
    static_assert(sizeof(T) == 4, "pin2: 32-bit values");
    if constexpr (N == 8)
        asm volatile("" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]),
                          "+v"(y[0]), "+v"(y[1]), "+v"(y[2]), "+v"(y[3]), "+v"(y[4]), "+v"(y[5]), "+v"(y[6]), "+v"(y[7]));
    else
        asm volatile("" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(y[0]), "+v"(y[1]), "+v"(y[2]), "+v"(y[3]));
}
template <class T, int N>
__device__ __forceinline__ void pin(T (&x)[N]) {
    if constexpr (sizeof(T) == 4) {
        if constexpr (N == 8)
            asm volatile("" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]));
        else
            asm volatile("" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]));
    } else {
        if constexpr (N == 8)
            asm volatile("" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]));
        else
            asm volatile("" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]));
    }
}

typedef int i32x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float byte_of(uint32_t w, int b) { return (float)((w >> (8 * b)) & 0xFFu); }

// n / d by FastDiv (dct3d_kernels.h): exact for n < 2^31 (cube indices are < 2^28)
__device__ __forceinline__ uint32_t fdiv(uint32_t n, FastDiv f) { return (uint32_t)(((uint64_t)n * f.m) >> f.s); }

}  // namespace dct3d
