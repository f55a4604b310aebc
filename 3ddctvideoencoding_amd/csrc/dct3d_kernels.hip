// dct3d_kernels.hip -- CDNA4 (gfx950) kernels of the 3D-DCT hot path.
//
// Work decomposition.  The 8x8x4 encode (and the 8-lane 8x8x8 form, variant 1): one wave64 owns 8
// cubes, 8 lanes per cube.
//   "row layout"  lane (c, y)        holds a[z][x]   (D x 8 values): the cube's row y of every frame
//   "face layout" lane (c, kz[,h])   holds b[y][x]   (8 x 8 or 8 x 4 values): one z-face (or half)
// The default 8x8x8 encode (encode16_kernel), the decode and the float drop-ins: 16 lanes per cube
// (2 D lanes for 8x8x4 decode), 32 values per lane, the permlane16 pair (l, l ^ 16) splitting each cube
// (DecGeom; encode16_kernel's comment has its three layouts).
// Two of the three separable 8-point passes run in registers in one layout, the third in the other;
// the single layout change is a wave-private LDS transpose (no workgroup barrier: one wave writes
// and reads its own region, LDS ops of a wave execute in order).  Cube-major int32 / fp64 traffic is
// staged through the same LDS region so every global access of the wave is a contiguous 1 KiB
// (16 B per lane) burst; the u8 raster side is 8 B per lane, 8 rows x 64 B per instruction.
//
// Encode (raster u8 -> quantised int32 cube-major), fp32, certified:
//   load rows (row layout) -> cube sum S, mean m, A = max|x - m| (xor-shuffles over the 8 lanes)
//   -> pass X (exact integer front, centring folded into X0) -> pass Z -> LDS transpose
//   -> pass Y (face layout) -> quantise: q = v * fp32(1/step), n = rint(q), certify |q - n| < thr_s
//   where thr_s = 0.5 - (A*G_s + E_s) (dct3d_plan.cpp) -> LDS staging -> 1 KiB coalesced stores.
//   DC = JavaRound(fp64(S) * coef_dc) exactly (the Java fold of the single DC group).
//   Uncertified coefficients are appended to a flag list; encode_fixup_kernel replays the Java fold.
// Decode (quantised int32 cube-major -> raster u8), fp64, certified:
//   staged 1 KiB loads -> face layout -> dequantise -> inverse pass Y -> LDS transpose (4 quarter
//   rounds, 16 B per lane-slot) -> inverse pass X -> inverse pass Z -> certify (no integer within
//   the bound of the pixel value in [1,255]) -> clamp, truncate (Decoder.java:112) -> 8 B row stores.
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

__device__ __forceinline__ float byte_of(uint32_t w, int b) { return (float)((w >> (8 * b)) & 0xFFu); }

// n / d by FastDiv (dct3d_kernels.h): exact for n < 2^31 (cube indices are < 2^28)
__device__ __forceinline__ uint32_t fdiv(uint32_t n, FastDiv f) { return (uint32_t)(((uint64_t)n * f.m) >> f.s); }

// =============================================================================================
// Fused encode
// =============================================================================================
// Loads row y = j of frames 0..D-1 of cube g (row layout).
typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
template <int D, bool NTL = false>
__device__ __forceinline__ void load_rows(const EncodeParams& P, uint32_t g, bool valid, int j, uint2 (&raw)[D]) {
    if (valid) {
        const uint32_t s = fdiv(g, P.div_cps);
        const uint32_t r = g - s * P.cubes_per_stack;
        const uint32_t by = fdiv(r, P.div_nbx), bx = r - by * P.nbx;
        const uint8_t* src = P.raster + (size_t)s * P.stack_stride + (size_t)(by * 8 + j) * P.width + bx * 8;
#pragma unroll
        for (int z = 0; z < D; z++) {
            if constexpr (NTL) {
                const u32x2_t t = __builtin_nontemporal_load((const u32x2_t*)(src + (size_t)z * P.plane));
                raw[z] = make_uint2(t.x, t.y);
            } else {
                raw[z] = *(const uint2*)(src + (size_t)z * P.plane);
            }
        }
    } else {
#pragma unroll
        for (int z = 0; z < D; z++) raw[z] = make_uint2(0u, 0u);
    }
}

template <int D>
__device__ __forceinline__ void to_float(const uint2 (&raw)[D], float (&a)[D][8]) {
#pragma unroll
    for (int z = 0; z < D; z++)
#pragma unroll
        for (int e = 0; e < 4; e++) {
            a[z][e] = byte_of(raw[z].x, e);
            a[z][e + 4] = byte_of(raw[z].y, e);
        }
}

// Cube statistics over the 8 lanes of a cube: S = sum, m = integer mean, A = max |x - m|.
// min/max on the float bit patterns (non-negative floats order like integers): v_max3/v_min3_u32.
template <int D>
__device__ __forceinline__ void cube_stats(const uint2 (&raw)[D], const float (&a)[D][8], uint32_t& S, int& m,
                                           float& A) {
    constexpr int CS = 64 * D;
    S = 0;
    uint32_t mx = 0u, mn = 0x7F800000u;
#pragma unroll
    for (int z = 0; z < D; z++) {
        S = __builtin_amdgcn_udot4(raw[z].x, 0x01010101u, S, false);
        S = __builtin_amdgcn_udot4(raw[z].y, 0x01010101u, S, false);
#pragma unroll
        for (int x = 0; x < 8; x += 2) {
            const uint32_t u0 = __float_as_uint(a[z][x]), u1 = __float_as_uint(a[z][x + 1]);
            asm("v_max3_u32 %0, %1, %2, %3" : "=v"(mx) : "v"(mx), "v"(u0), "v"(u1));
            asm("v_min3_u32 %0, %1, %2, %3" : "=v"(mn) : "v"(mn), "v"(u0), "v"(u1));
        }
    }
#pragma unroll
    for (int o = 1; o < 8; o <<= 1) {
        S += __shfl_xor(S, o, 64);
        mx = max(mx, (uint32_t)__shfl_xor((int)mx, o, 64));
        mn = min(mn, (uint32_t)__shfl_xor((int)mn, o, 64));
    }
    m = (int)((S + CS / 2) / CS);
    const float mf = (float)m;
    A = fmaxf(__uint_as_float(mx) - mf, mf - __uint_as_float(mn));  // exact (small integers)
}

// Forward transform of the wave's 8 cubes: row layout a[z][x] -> face layout coefficients b[ky][kx'].
// Uses the wave's LDS region (no cross-wave sharing).
template <int D, int NB>
__device__ __forceinline__ void forward_cube(float (&a)[D][8], int m, int c, int j, char* wl, float (&b)[8][NB]) {
    const float dcsub = 8.0f * (float)m;
    // pass X (integer front exact, cube-mean centring folded into X0), pass Z
    pin(a[0]);
#pragma unroll
    for (int z = 0; z < D; z++) {
        fdct8<true, true>(a[z], dcsub);
        if (z + 1 < D) pin2(a[z], a[z + 1]);
        else pin(a[z]);
    }
    {
        float col[8][D];
#pragma unroll
        for (int x = 0; x < 8; x++)
#pragma unroll
            for (int z = 0; z < D; z++) col[x][z] = a[z][x];
#pragma unroll
        for (int x = 0; x < 8; x++) {
            fdctN<D, false, false>(col[x], 0.f);
            if (x < 7) pin2(col[x], col[x + 1]);
            else pin(col[x]);
        }
#pragma unroll
        for (int x = 0; x < 8; x++)
#pragma unroll
            for (int z = 0; z < D; z++) a[z][x] = col[x][z];
    }
    // LDS transpose: row layout (c, y)[kz][x] -> face layout (c, j)[y][kx']
    if constexpr (D == 8) {
#pragma unroll
        for (int h = 0; h < 2; h++) {
#pragma unroll
            for (int kz = 0; kz < 8; kz++)
                *(float4*)(wl + (c * 8 + kz) * kSlot + j * 16) =
                    make_float4(a[kz][4 * h], a[kz][4 * h + 1], a[kz][4 * h + 2], a[kz][4 * h + 3]);
            wave_lds_sync();
#pragma unroll
            for (int y = 0; y < 8; y++) {
                float4 t = *(const float4*)(wl + (c * 8 + j) * kSlot + y * 16);
                b[y][4 * h] = t.x; b[y][4 * h + 1] = t.y; b[y][4 * h + 2] = t.z; b[y][4 * h + 3] = t.w;
            }
            wave_lds_sync();
        }
    } else {
        // two rounds (x halves h): every lane writes its rows' half h; the lanes owning kx half h read
#pragma unroll
        for (int h = 0; h < 2; h++) {
#pragma unroll
            for (int kz = 0; kz < 4; kz++)
                *(float4*)(wl + (c * 4 + kz) * kSlot + j * 16) =
                    make_float4(a[kz][4 * h], a[kz][4 * h + 1], a[kz][4 * h + 2], a[kz][4 * h + 3]);
            wave_lds_sync();
            if ((j & 1) == h) {
#pragma unroll
                for (int y = 0; y < 8; y++) {
                    float4 t = *(const float4*)(wl + (c * 4 + (j >> 1)) * kSlot + y * 16);
                    b[y][0] = t.x; b[y][1] = t.y; b[y][2] = t.z; b[y][3] = t.w;
                }
            }
            wave_lds_sync();
        }
    }
    // pass Y
    {
        float col[NB][8];
#pragma unroll
        for (int x = 0; x < NB; x++)
#pragma unroll
            for (int y = 0; y < 8; y++) col[x][y] = b[y][x];
        pin(col[0]);
#pragma unroll
        for (int x = 0; x < NB; x++) {
            fdct8<false, false>(col[x], 0.f);
            if (x + 1 < NB) pin2(col[x], col[x + 1]);
            else pin(col[x]);
        }
#pragma unroll
        for (int x = 0; x < NB; x++)
#pragma unroll
            for (int y = 0; y < 8; y++) b[y][x] = col[x][y];
    }
}

typedef int i32x4_t __attribute__((ext_vector_type(4)));
template <bool NT>
__device__ __forceinline__ void store16(void* p, const int4& v) {
    if constexpr (NT) {
        i32x4_t t = {v.x, v.y, v.z, v.w};
        __builtin_nontemporal_store(t, (i32x4_t*)p);
    } else {
        *(int4*)p = v;
    }
}

// Stage the wave's 8 quantised cubes through LDS (face-padded cube-major) and store them 1 KiB per
// instruction (lane (c, j) holds qv[ky][kx'] of cube c, kz = j (8x8x8) / j >> 1 (8x8x4)).
template <int D, bool NT>
__device__ __forceinline__ void enc_stage_store(const EncodeParams& P, const int32_t (&qv)[8][(D == 8) ? 8 : 4],
                                                char* wl, int lane, uint32_t cube0) {
    constexpr int CS = 64 * D;
    const int c = lane >> 3, j = lane & 7;
    const int kz = (D == 8) ? j : (j >> 1);
    constexpr int ROUNDS = 2;
    constexpr int CUBES_PER_ROUND = 8 / ROUNDS;
    constexpr int CHUNK_ITERS = CUBES_PER_ROUND * (CS / 4) / 64;  // 16-byte chunks per lane per round
#pragma unroll
    for (int rd = 0; rd < ROUNDS; rd++) {
        if ((c / CUBES_PER_ROUND) == rd) {
            const int cc = c % CUBES_PER_ROUND;
            if constexpr (D == 8) {
#pragma unroll
                for (int ky = 0; ky < 8; ky++)
#pragma unroll
                    for (int h = 0; h < 2; h++)
                        *(int4*)(wl + (cc * 8 + kz) * kFace + ky * 32 + h * 16) =
                            make_int4(qv[ky][4 * h], qv[ky][4 * h + 1], qv[ky][4 * h + 2], qv[ky][4 * h + 3]);
            } else {
#pragma unroll
                for (int ky = 0; ky < 8; ky++)
                    *(int4*)(wl + (cc * 4 + kz) * kFace + ky * 32 + (j & 1) * 16) =
                        make_int4(qv[ky][0], qv[ky][1], qv[ky][2], qv[ky][3]);
            }
        }
        wave_lds_sync();
        const uint32_t rcube0 = cube0 + rd * CUBES_PER_ROUND;
        char* outb = (char*)(P.out + (size_t)rcube0 * CS);
#pragma unroll
        for (int t = 0; t < CHUNK_ITERS; t++) {
            const int q = t * 64 + lane;                 // 16-byte chunk within the round
            const int cc = q / (CS / 4);                 // CS*4 bytes per cube = CS/4 chunks
            const int face = (q >> 4) % D;
            const int w = q & 15;
            if (rcube0 + cc < P.n_cubes) {
                const int4 v = *(const int4*)(wl + (cc * D + face) * kFace + w * 16);
                store16<NT>(outb + (size_t)q * 16, v);
            }
        }
        wave_lds_sync();
    }

}

// The quantise/certify tables in LDS as {1/step_s, G_s, 0.5 - E_s, 0} (s = kx + ky + kz < 22), one copy
// per block at a fixed LDS address (no base register to keep live across the transform): LDS reads
// instead of three global loads per sum waited on after the transform.  EVERY wave writes the whole
// table right after its row loads (identical bits, so the other waves' writes change nothing) and
// reads only after its own writes (one wave's LDS operations complete in order).
constexpr int kTabN = 24;
__device__ __forceinline__ void enc_tables(const EncodeParams& P, float4* tab, int lane) {
    if (lane < kTabN) tab[lane] = make_float4(P.tab_rstep[lane], P.tab_G[lane], 0.5f - P.tab_E[lane], 0.f);
}
// Row ky of the quantise loop uses sums sz + ky .. sz + ky + NB - 1: the window slides by one entry per
// row, read at the row's start (the opaque sz keeps the reads there), so 2 NB table registers are live
// instead of 2 NI.
template <int NB, int NI>
__device__ __forceinline__ void tab_window(const float4* tab, int& sz, int ky, float A, float (&rr)[NI],
                                           float (&thr)[NI]) {
    asm volatile("" : "+v"(sz));
    const int lo = ky == 0 ? 0 : ky + NB - 1;
#pragma unroll
    for (int i = lo; i < ky + NB; i++) {
        const float* t = (const float*)(tab + sz + i);
        rr[i] = t[0];
        thr[i] = __builtin_fmaf(-A, t[1], t[2]);
    }
}

// Everything after the row loads, for the 8 cubes from cube0: statistics, transform, quantise +
// certify, staged 1 KiB stores, uncertified coefficients to the flag list.
template <int D, bool NT>
__device__ __forceinline__ void encode_body(const EncodeParams& P, const uint2 (&raw)[D], char* wl,
                                            const float4* tab, int lane, uint32_t cube0) {
    constexpr int CS = 64 * D;
    constexpr int NB = (D == 8) ? 8 : 4;      // kx values per lane in the face layout
    constexpr int NI = 7 + NB;                // distinct (ky + kx') sums per lane
    const int c = lane >> 3, j = lane & 7;
    const int kz = (D == 8) ? j : (j >> 1);
    const int kx0 = (D == 8) ? 0 : (j & 1) * 4;
    const int so = kz + kx0;
    const uint32_t g = cube0 + c;
    const bool valid = g < P.n_cubes;

    float a[D][8];
    to_float<D>(raw, a);
    uint32_t S;
    int m;
    float A;
    cube_stats<D>(raw, a, S, m, A);
    asm volatile("" : "+v"(S), "+v"(m), "+v"(A));  // stats now: raw dies after conversion

    float b[8][NB];
    forward_cube<D, NB>(a, m, c, j, wl, b);

    // ---- quantise + certify (thr_s = 0.5 - (A*G_s + E_s), dct3d_plan.cpp) ----
    // The per-lane tables are read row by row from the block's LDS copy (enc_tables, tab_window).
    int sz = so;
    float rr[NI], thr[NI];
    // Uncertified coefficients: 8x8x4 (INL) appends them to the flag list inside the row loop while
    // q is in registers -- its exact ties (the 4-point k = 2 row is +-1/2) flag a quarter of the
    // waves; 8x8x8 (flags in ~5 % of waves, registers at the 128 limit) re-derives them after the
    // stores from reloaded rows instead.
    constexpr bool INL = (D == 4);
    int32_t qv[8][NB];
    int overflow = 0, flag = 0;
#pragma unroll
    for (int ky = 0; ky < 8; ky++) {
        pin(b[ky]);
        tab_window<NB, NI>(tab, sz, ky, A, rr, thr);
        bool f = false;
        float qq[NB];
#pragma unroll
        for (int x = 0; x < NB; x++) {
            qq[x] = b[ky][x] * rr[ky + x];
            const float n = __builtin_rintf(qq[x]);
            f |= __builtin_fabsf(qq[x] - n) >= thr[ky + x];
            qv[ky][x] = (int32_t)n;
        }
        if (!INL) flag |= (int)f;
        if (INL && __builtin_expect(f && valid, 0)) {
#pragma unroll
            for (int x = 0; x < NB; x++)
                if (__builtin_fabsf(qq[x] - __builtin_rintf(qq[x])) >= thr[ky + x]) {
                    const uint32_t k = (uint32_t)((kz * 8 + ky) * 8 + kx0 + x);
                    const uint32_t idx = atomicAdd(&P.counters[0], 1u);
                    if (idx < P.flag_cap) P.flag_list[idx] = (unsigned long long)g * CS + k;
                    else overflow = 1;
                }
        }
        pin(qv[ky]);
        asm volatile("" : "+v"(overflow), "+v"(flag));  // the row's checks complete here (q, n die)
    }
    if (j == 0) qv[0][0] = java_round_dev((double)S * P.coef_dc);  // exact DC (single Java group)

    enc_stage_store<D, NT>(P, qv, wl, lane, cube0);

    // ---- !INL rare path: identify uncertified coefficients (recomputed from reloaded rows) ----
    if (!INL && __builtin_expect(__ballot(flag && valid) != 0ull, 0)) {
        uint2 raw2[D];
        load_rows<D>(P, g, valid, j, raw2);
        float a2[D][8];
        to_float<D>(raw2, a2);
        float b2[8][NB];
        forward_cube<D, NB>(a2, m, c, j, wl, b2);
        if (flag && valid) {
#pragma unroll
            for (int ky = 0; ky < 8; ky++)
#pragma unroll
                for (int x = 0; x < NB; x++) {
                    const float th2 = __builtin_fmaf(-A, P.tab_G[so + ky + x], 0.5f - P.tab_E[so + ky + x]);
                    const float q = b2[ky][x] * rr[ky + x];
                    const float n = __builtin_rintf(q);
                    if (__builtin_fabsf(q - n) >= th2) {
                        const uint32_t k = (uint32_t)((kz * 8 + ky) * 8 + kx0 + x);
                        const uint32_t idx = atomicAdd(&P.counters[0], 1u);
                        if (idx < P.flag_cap) P.flag_list[idx] = (unsigned long long)g * CS + k;
                        else overflow = 1;
                    }
                }
        }
        wave_lds_sync();
    }
    // ---- flag-list overflow: the cube goes to the whole-cube replay (one entry per cube) ----
    const unsigned long long ov = __ballot(overflow != 0);
    if (__builtin_expect(ov != 0ull, 0)) {
        const uint32_t mine = (uint32_t)(ov >> (c * 8)) & 0xFFu;
        if (overflow && (__builtin_ctz(mine) == j)) {
            const uint32_t idx = atomicAdd(&P.counters[1], 1u);
            P.cube_list[idx] = g;  // capacity n_cubes: never overflows
        }
    }

}

// One wave = one group of 8 consecutive cubes (register-prefetch loops over several groups spill
// and were 25-40 % slower: profiles/r01/encode_variant_sweep.txt).
template <int D, bool NT, bool NTL = false>
__global__ __launch_bounds__(kBlock, 4) void encode_kernel(EncodeParams P) {
    __shared__ __attribute__((aligned(16))) char lds[kWavesPerBlock * enc_wave_lds<D>()];
    __shared__ float4 s_tab[kTabN];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t cube0 = P.g_base + (blockIdx.x * kWavesPerBlock + wave) * kCubesPerWave;
    uint2 raw[D];
    load_rows<D, NTL>(P, cube0 + (lane >> 3), cube0 + (lane >> 3) < P.n_cubes, lane & 7, raw);  // in flight first
    if (cube0 >= P.n_cubes) return;  // wave-uniform
    enc_tables(P, s_tab, lane);
    encode_body<D, NT>(P, raw, lds + wave * enc_wave_lds<D>(), s_tab, lane, cube0);
}

// =============================================================================================
// Exact Java fold for flagged (cube, k): out = JavaRound(fold_g(S_g * coef_g) / step)
// =============================================================================================
// The Java fold of DCT.java:44-52 for coefficient k of cube g, by one whole wave:
//   out = sum over groups gi (HashMap order) of  S_gi * coef_gi,  S_gi = exact integer pixel sums.
// Group sums: LDS integer atomics (exact).  Products: one lane per group, in parallel (each is one
// correctly rounded fp64 multiply, as in Java).  The fold itself (the only order-dependent part) runs
// on lane 0 over the products in LDS.  ssum / prod: the wave's kMaxGroupsDev-entry scratch.  The
// result is valid in lane 0.
struct ReplayGeom {
    const uint8_t* raster;
    uint32_t cubes_per_stack, nbx, width;
    uint64_t plane, stack_stride;
    const int32_t* ngroups;
    const double* coef;
    const uint8_t* group_of;
};
// The global loads of one replay (split from the fold so that a caller can issue them early: on gfx9
// a load issued after a wave's stores waits for those stores too, vmcnt being one in-order counter).
struct ReplayIn {
    int ng;
    double cf;
    uint2 px, gr;
};
template <int D>
__device__ __forceinline__ ReplayIn replay_load(const ReplayGeom& R, uint32_t g, uint32_t k, int lane) {
    constexpr int CS = 64 * D;
    ReplayIn in;
    in.ng = R.ngroups[k];
    in.cf = R.coef[(size_t)k * kMaxGroupsDev + lane];  // lanes >= ng: unused
    in.px = in.gr = make_uint2(0u, 0u);
    if (lane * 8 < CS) {
        const int z = lane >> 3, y = lane & 7;
        const uint32_t s = g / R.cubes_per_stack;
        const uint32_t r = g - s * R.cubes_per_stack;
        const uint32_t by = r / R.nbx, bx = r - by * R.nbx;
        const uint8_t* src = R.raster + (size_t)s * R.stack_stride + (size_t)z * R.plane +
                             (size_t)(by * 8 + y) * R.width + bx * 8;
        in.px = *(const uint2*)src;
        in.gr = *(const uint2*)(R.group_of + (size_t)k * CS + lane * 8);
    }
    return in;
}
// LEAN: the fold loop is not unrolled (in-wave replay: its registers would count against the main path)
template <int D, bool LEAN = false>
__device__ __forceinline__ int replay_fold(const ReplayIn& in, uint32_t k, int lane, int* ssum, double* prod) {
    constexpr int CS = 64 * D;
    ssum[lane] = 0;
    wave_lds_sync();
    if (lane * 8 < CS) {
#pragma unroll
        for (int bb = 0; bb < 4; bb++) {
            const uint32_t g0 = (in.gr.x >> (8 * bb)) & 0xFF, g1 = (in.gr.y >> (8 * bb)) & 0xFF;
            if (g0 < kMaxGroupsDev) atomicAdd(&ssum[g0], (int)((in.px.x >> (8 * bb)) & 0xFF));
            if (g1 < kMaxGroupsDev) atomicAdd(&ssum[g1], (int)((in.px.y >> (8 * bb)) & 0xFF));
        }
    }
    wave_lds_sync();
    prod[lane] = __dmul_rn((double)ssum[lane], lane < in.ng ? in.cf : 0.0);
    wave_lds_sync();
    int q = 0;
    if (lane == 0) {
        const int ng = in.ng;
        double acc = 0.0;
        int gi = 0;
        if constexpr (LEAN) {
#pragma unroll 1
            for (; gi + 4 <= ng; gi += 4) {  // DCT.java:50, output += sum * coefficient, in order
                const double p0 = prod[gi], p1 = prod[gi + 1], p2 = prod[gi + 2], p3 = prod[gi + 3];
                acc = __dadd_rn(__dadd_rn(__dadd_rn(__dadd_rn(acc, p0), p1), p2), p3);
            }
        } else {
            for (; gi + 4 <= ng; gi += 4) {
                const double p0 = prod[gi], p1 = prod[gi + 1], p2 = prod[gi + 2], p3 = prod[gi + 3];
                acc = __dadd_rn(__dadd_rn(__dadd_rn(__dadd_rn(acc, p0), p1), p2), p3);
            }
        }
#pragma unroll 1
        for (; gi < ng; gi++) acc = __dadd_rn(acc, prod[gi]);
        const int kz = k / 64, ky = (k / 8) & 7, kx = k & 7;
        const int st = max(1, 5 * (kx + ky + kz));
        q = java_round_dev(__ddiv_rn(acc, (double)st));
    }
    wave_lds_sync();
    return q;
}
template <int D>
__device__ __forceinline__ int exact_coef(const ReplayGeom& R, uint32_t g, uint32_t k, int lane, int* ssum,
                                          double* prod) {
    return replay_fold<D>(replay_load<D>(R, g, k, lane), k, lane, ssum, prod);
}

// ---------------------------------------------------------------------------------------------
// Encode, 16 lanes per cube (8x8x8): the decode's geometry in the forward direction.  Lane (c, k, h)
// of the wave's 4 cubes: c = (lane >> 5) * 2 + ((lane & 15) >> 3), k = lane & 7, h = (lane >> 4) & 1
// (a cube's lanes are the permlane16 pairs (l, l ^ 16)).
//   rows  a[r][x]: row y = k of frame z = 4h + r                           4 lines along x: pass X
//   swap  of the pair's off-diagonal 4x4 blocks: x = 4h + e, z = r in a[r][e], z = 4 + r in a[r][4 + e]
//                                                                          4 lines along z: pass Z
//   LDS   (two y halves) -> lane (c, kz = k, h): b[y][e], x = 4h + e       4 lines along y: pass Y
//   quantise coefficient (kz = k, ky, kx = 4h + e): s = k + 4h + ky + e
// Per line these are exactly encode_kernel's butterflies, in the same pass order (X, Z, Y): the
// values, and so the certification bounds, are identical.  32 floats per lane instead of 64, 4.5 KiB
// of LDS per wave: more waves per CU to hide each wave's transform latency.
constexpr int kE16CPW = 4;     // cubes per wave
constexpr int kE16TZ = 144;    // transpose: kz stride (4 y x 16 B per h, 2 h, + 16 B: bank spread)
constexpr int kE16TC = 8 * kE16TZ;
constexpr int kE16SC = 8 * kFace;  // output staging: cube stride (faces of 256 + 16 B)
constexpr int kE16Lds = 4 * kE16TC;
static_assert(kE16Lds >= 2 * kE16SC, "two staged cubes per round");

// rows of the lane's cube (row y = k of frames 4h .. 4h + 3), zero past the end
__device__ __forceinline__ void e16_load(const EncodeParams& P, uint32_t g, bool valid, int k, int h, uint2 (&raw)[4]) {
    if (valid) {
        const uint32_t st = fdiv(g, P.div_cps);
        const uint32_t rr = g - st * P.cubes_per_stack;
        const uint32_t by = fdiv(rr, P.div_nbx), bx = rr - by * P.nbx;
        const uint8_t* src = P.raster + (size_t)st * P.stack_stride + (size_t)(by * 8 + k) * P.width + bx * 8 +
                             (size_t)(4 * h) * P.plane;
#pragma unroll
        for (int r = 0; r < 4; r++) raw[r] = *(const uint2*)(src + (size_t)r * P.plane);
    } else {
#pragma unroll
        for (int r = 0; r < 4; r++) raw[r] = make_uint2(0u, 0u);
    }
}

// Statistics, passes X / Z / Y, quantise + certify, exact DC.  Uncertified coefficients are returned
// as the lane's mask fm (bit 4 ky + e: coefficient (kz = k, ky, kx = 4h + e)); the caller replays them.
__device__ __forceinline__ void e16_body(const EncodeParams& P, const uint2 (&raw)[4], char* wl, const float4* tab,
                                         int lane, bool valid, int32_t (&qv)[8][4], uint32_t& fm) {
    constexpr int CS = 512;
    const int k = lane & 7, h = (lane >> 4) & 1;
    const int c = (lane >> 5) * 2 + ((lane & 15) >> 3);
    // ---- statistics over the cube's 16 lanes: S, m, A (as cube_stats) ----
    float a[4][8];
#pragma unroll
    for (int r = 0; r < 4; r++)
#pragma unroll
        for (int e = 0; e < 4; e++) {
            a[r][e] = byte_of(raw[r].x, e);
            a[r][e + 4] = byte_of(raw[r].y, e);
        }
    uint32_t S = 0, mx = 0u, mn = 0x7F800000u;
#pragma unroll
    for (int r = 0; r < 4; r++) {
        S = __builtin_amdgcn_udot4(raw[r].x, 0x01010101u, S, false);
        S = __builtin_amdgcn_udot4(raw[r].y, 0x01010101u, S, false);
#pragma unroll
        for (int x = 0; x < 8; x += 2) {
            const uint32_t u0 = __float_as_uint(a[r][x]), u1 = __float_as_uint(a[r][x + 1]);
            asm("v_max3_u32 %0, %1, %2, %3" : "=v"(mx) : "v"(mx), "v"(u0), "v"(u1));
            asm("v_min3_u32 %0, %1, %2, %3" : "=v"(mn) : "v"(mn), "v"(u0), "v"(u1));
        }
    }
#pragma unroll
    for (int o = 1; o <= 16; o <<= 1) {
        if (o == 8) continue;  // the cube's lanes: k bits (1, 2, 4) and h (16)
        S += __shfl_xor(S, o, 64);
        mx = max(mx, (uint32_t)__shfl_xor((int)mx, o, 64));
        mn = min(mn, (uint32_t)__shfl_xor((int)mn, o, 64));
    }
    const int m = (int)((S + CS / 2) / CS);
    float A = fmaxf(__uint_as_float(mx) - (float)m, (float)m - __uint_as_float(mn));
    asm volatile("" : "+v"(S), "+v"(A));

    // ---- pass X (exact integer front, centring folded into X0) ----
    const float dcsub = 8.0f * (float)m;
    pin(a[0]);
#pragma unroll
    for (int r = 0; r < 4; r++) {
        fdct8<true, true>(a[r], dcsub);
        if (r + 1 < 4) pin2(a[r], a[r + 1]);
        else pin(a[r]);
    }
    // ---- swap the off-diagonal 4x4 blocks of the lane pair: lines along z ----
#pragma unroll
    for (int r = 0; r < 4; r++)
#pragma unroll
        for (int e = 0; e < 4; e++) {
            const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(a[r][e]), __float_as_uint(a[r][4 + e]),
                                                             false, false);
            a[r][e] = __uint_as_float((uint32_t)sw[0]);
            a[r][4 + e] = __uint_as_float((uint32_t)sw[1]);
        }
    // ---- pass Z: line e (x = 4h + e) = a[0..3][e], a[0..3][4 + e] ----
#pragma unroll
    for (int e = 0; e < 4; e++) {
        float col[8];
#pragma unroll
        for (int z = 0; z < 4; z++) {
            col[z] = a[z][e];
            col[4 + z] = a[z][4 + e];
        }
        pin(col);
        fdct8<false, false>(col, 0.f);
        pin(col);
#pragma unroll
        for (int z = 0; z < 4; z++) {
            a[z][e] = col[z];
            a[z][4 + e] = col[4 + z];
        }
    }
    // now coefficient kz of line e: a[kz][e] (kz < 4), a[kz - 4][4 + e]

    // ---- LDS transpose in two y halves: lane (c, y = k, h) -> lane (c, kz = k, h) ----
    float b[8][4];
#pragma unroll
    for (int rd = 0; rd < 2; rd++) {
        if ((k >> 2) == rd) {
            char* dst = wl + c * kE16TC + h * 64 + (k & 3) * 16;
#pragma unroll
            for (int kz = 0; kz < 8; kz++) {
                const float* v = kz < 4 ? &a[kz][0] : &a[kz - 4][4];
                *(float4*)(dst + kz * kE16TZ) = make_float4(v[0], v[1], v[2], v[3]);
            }
        }
        wave_lds_sync();
        const char* src = wl + c * kE16TC + k * kE16TZ + h * 64;
#pragma unroll
        for (int yy = 0; yy < 4; yy++) {
            const float4 t = *(const float4*)(src + yy * 16);
            b[4 * rd + yy][0] = t.x; b[4 * rd + yy][1] = t.y; b[4 * rd + yy][2] = t.z; b[4 * rd + yy][3] = t.w;
        }
        wave_lds_sync();
    }
    // ---- pass Y ----
#pragma unroll
    for (int e = 0; e < 4; e++) {
        float col[8];
#pragma unroll
        for (int y = 0; y < 8; y++) col[y] = b[y][e];
        pin(col);
        fdct8<false, false>(col, 0.f);
        pin(col);
#pragma unroll
        for (int y = 0; y < 8; y++) b[y][e] = col[y];
    }

    // ---- quantise + certify; uncertified coefficients recorded in fm while q is in registers ----
    int sz = k + 4 * h;
    float rr[11], thr[11];
    fm = 0u;
#pragma unroll
    for (int ky = 0; ky < 8; ky++) {
        pin(b[ky]);
        tab_window<4, 11>(tab, sz, ky, A, rr, thr);
#pragma unroll
        for (int e = 0; e < 4; e++) {
            const float qq = b[ky][e] * rr[ky + e];
            const float n = __builtin_rintf(qq);
            fm |= (__builtin_fabsf(qq - n) >= thr[ky + e] ? 1u : 0u) << (4 * ky + e);
            qv[ky][e] = (int32_t)n;
        }
        pin(qv[ky]);
        asm volatile("" : "+v"(fm));
    }
    if (k == 0 && h == 0) {
        qv[0][0] = java_round_dev((double)S * P.coef_dc);  // exact DC (the single Java group)
        fm &= ~1u;
    }
    if (!valid) fm = 0u;
}

// In-wave exact replay (encode16): the uncertified coefficient at bit `bit` of lane src's mask fm
// (bit 4 ky + e of lane (c, k, h): coefficient (kz = k, ky, kx = 4h + e) of cube cube0 + c).
__device__ __forceinline__ void e16_flag_pos(uint32_t fm, int src, uint32_t cube0, uint32_t& g, uint32_t& kk) {
    const int bit = __shfl(fm ? __builtin_ctz(fm) : 0, src, 64);
    const int sk = src & 7, sh = (src >> 4) & 1, sc = (src >> 5) * 2 + ((src & 15) >> 3);
    g = cube0 + sc;
    kk = (uint32_t)((sk * 8 + (bit >> 2)) * 8 + 4 * sh + (bit & 3));
}

// Second certificate (8x8x8 rare path): every coefficient the fp32 certificate left open (fm) is
// re-evaluated in fp64 from the cube's bytes, one coefficient per cube per round (a cube's 16 lanes
// together; the wave's 4 cubes in parallel):
//   v64 = sum over the cube's lanes (c, k, h) of  b[ky][k] * sum_e b[kz][4h+e] * sum_x x[4h+e][k][x] b[kx][x]
// (b = the fp64 basis, fma chains, an xor-butterfly sum: every lane of the cube gets the same bits).
// q64 = v64 / step is settled iff |q64 - rint(q64)| < thr64[s]: then Math.round of Java's value is
// rint(q64) (bound: dct3d_plan.cpp, "second certificate").  What stays open is returned in fm for the
// exact Java fold; nset counts the settled ones (owner lanes).
// Timing: the rows (raw, again: L2) and the tables (bv, tv) were loaded before the wave's stores and
// arrive while those drain; this runs after the stores, and the owning lane writes a settled value
// over the provisional one once the wave's stores are complete (vmcnt(0): the same word was stored by
// another lane of the wave).  Register pressure stays with the main path's 72 VGPRs.  s_b: the block's
// copy of the tables ([64] basis, [32] thresholds), written by every wave that takes this path
// (identical bits) and read only after its own writes.
__device__ __forceinline__ void e16_recheck64(const EncodeParams& P, const uint2 (&raw)[4], double bv, double tv,
                                              double* s_b, int lane, uint32_t cube0, uint32_t& fm, uint32_t& nset) {
    constexpr int CS = 512;
    const int k = lane & 7, h = (lane >> 4) & 1;
    s_b[lane] = bv;
    if (lane < 32) s_b[64 + lane] = tv;
    wave_lds_sync();
    const int base = (lane & 32) + (lane & 8);
    const uint64_t cmask = (0xFFull << base) | (0xFFull << (base + 16));  // this lane's cube
    uint32_t open = 0u;
    nset = 0u;
    for (;;) {
        const uint64_t any = __ballot(fm != 0u);
        if (any == 0ull) break;
        const uint64_t mine = any & cmask;
        const int src = mine ? (int)__builtin_ctzll(mine) : lane;
        const int bit = __shfl(fm ? (int)__builtin_ctz(fm) : 0, src, 64);
        const int kz = src & 7, ky = bit >> 2, kx = 4 * ((src >> 4) & 1) + (bit & 3);
        const double* bx = s_b + kx * 8;
        double t = 0.0;
#pragma unroll 1
        for (int e = 0; e < 4; e += 2) {  // two rows' chains side by side
            uint32_t w[4] = {raw[e].x, raw[e + 1].x, raw[e].y, raw[e + 1].y};
            double r0 = 0.0, r1 = 0.0;
#pragma unroll
            for (int x = 0; x < 8; x++) {
                const int i = x >> 2;
                const double b = bx[x];
                r0 = __fma_rn((double)(w[2 * i] & 0xFFu), b, r0);
                r1 = __fma_rn((double)(w[2 * i + 1] & 0xFFu), b, r1);
                w[2 * i] >>= 8;
                w[2 * i + 1] >>= 8;
                asm volatile("" : "+v"(w[2 * i]), "+v"(w[2 * i + 1]));  // conversions stay in the chains
            }
            t = __fma_rn(r0, s_b[kz * 8 + 4 * h + e], t);
            t = __fma_rn(r1, s_b[kz * 8 + 4 * h + e + 1], t);
        }
        t = __dmul_rn(t, s_b[ky * 8 + k]);
#pragma unroll
        for (int o = 1; o <= 16; o <<= 1) {
            if (o == 8) continue;  // the cube's lanes: k bits (1, 2, 4) and h (16)
            t = __dadd_rn(t, __shfl_xor(t, o, 64));
        }
        if (mine != 0ull && lane == src) {
            const int s = kz + ky + kx;
            const double q = __ddiv_rn(t, (double)(5 * s));  // s >= 1: the DC is never open
            const double n = __builtin_rint(q);
            if (__builtin_fabs(q - n) < s_b[64 + s]) {
                const uint32_t cube = cube0 + (lane >> 5) * 2 + ((lane & 15) >> 3);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                P.out[(size_t)cube * CS + (kz * 8 + ky) * 8 + kx] = (int32_t)n;
                nset++;
            } else {
                open |= 1u << bit;
            }
            fm &= fm - 1u;  // its lowest bit is `bit`
        }
    }
    fm = open;
    wave_lds_sync();
}

// MEM (dct3d_encode_memonly_dev, DIAGNOSTIC: the output is NOT a DCT): the same loads, staging and
// stores with the transform, quantisation and certification replaced by a few integer ops.
// One launch is the whole encode: no flag list, no counter reset, no fixup launch.  Block 0 zeroes the
// next call's counter slot (P.replay_clear; the two slots alternate between calls).  7 waves per SIMD
// (72 VGPRs) is what the main path needs; the attribute keeps the rare paths from raising it (they
// spill a few registers to scratch instead, off the main path).
static_assert(kMaxGroupsDev * (4 + 8) <= kE16Lds, "exact-replay scratch fits the wave's region");
template <bool NT, bool MEM = false>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(7))) void encode16_kernel(EncodeParams P) {
    constexpr int CS = 512;
    __shared__ __attribute__((aligned(16))) char lds[kWavesPerBlock * kE16Lds];
    __shared__ float4 s_tab[kTabN];
    __shared__ double s_b64[96];  // second certificate tables (rare path)
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t cube0 = P.g_base + (blockIdx.x * kWavesPerBlock + wave) * kE16CPW;
    const int k = lane & 7, h = (lane >> 4) & 1;
    const int c = (lane >> 5) * 2 + ((lane & 15) >> 3);
    const uint32_t g = cube0 + c;
    const bool valid = g < P.n_cubes;
    uint2 raw[4];
    e16_load(P, g, valid, k, h, raw);
    if (!MEM && blockIdx.x == 0 && P.replay_clear) {
#pragma unroll
        for (int i = 0; i < 2 * kCountSpread / kBlock; i++) P.replay_clear[i * kBlock + threadIdx.x] = 0u;
    }
    if (cube0 >= P.n_cubes) return;  // wave-uniform
    char* wl = lds + wave * kE16Lds;
    int32_t qv[8][4];
    uint32_t fm = 0u;
    if constexpr (MEM) {
#pragma unroll
        for (int ky = 0; ky < 8; ky++)
#pragma unroll
            for (int e = 0; e < 4; e++) qv[ky][e] = (int32_t)(((ky & 1) ? raw[e].y : raw[e].x) >> (ky * 3 % 24)) & 255;
    } else {
        enc_tables(P, s_tab, lane);
        e16_body(P, raw, wl, s_tab, lane, valid, qv, fm);
    }
    // ---- rare path, part 1: the second certificate's loads, issued before the stores (a load issued
    //      after them would wait for them too: one in-order vmcnt) ----
    const bool rare = !MEM && P.recheck && __builtin_expect(__ballot(fm != 0u) != 0ull, 0);  // wave-uniform
    uint2 raw2[4];
    double bv = 0.0, tv = 0.0;
    if (rare) {
        e16_load(P, g, valid, k, h, raw2);
        bv = P.tab64[lane];
        tv = lane < 32 ? P.tab64[64 + lane] : 0.0;
    }

    const ReplayGeom R{P.raster, P.cubes_per_stack, P.nbx, P.width, P.plane, P.stack_stride,
                       P.ngroups, P.coef, P.group_of};

    // ---- stage two cubes per round (lanes 0-31: cubes 0, 1; lanes 32-63: cubes 2, 3), 1 KiB stores ----
#pragma unroll
    for (int rd = 0; rd < 2; rd++) {
        if ((lane >> 5) == rd) {
            char* dst = wl + (c & 1) * kE16SC + k * kFace + h * 16;
#pragma unroll
            for (int ky = 0; ky < 8; ky++)
                *(int4*)(dst + ky * 32) = make_int4(qv[ky][0], qv[ky][1], qv[ky][2], qv[ky][3]);
        }
        wave_lds_sync();
        const uint32_t rcube0 = cube0 + 2 * rd;
        char* outb = (char*)(P.out + (size_t)rcube0 * CS);
#pragma unroll
        for (int t = 0; t < 4; t++) {
            const int q = t * 64 + lane;  // 16-byte chunk of the round's two cubes
            const int cc = q >> 7, face = (q >> 4) & 7, w = q & 15;
            if (rcube0 + cc < P.n_cubes) {
                const int4 v = *(const int4*)(wl + cc * kE16SC + face * kFace + w * 16);
                store16<NT>(outb + (size_t)q * 16, v);
            }
        }
        wave_lds_sync();
    }

    // ---- rare path, part 2: the second certificate (one counter update per wave) ----
    if (rare) {
        uint32_t nset;
        e16_recheck64(P, raw2, bv, tv, s_b64, lane, cube0, fm, nset);
        for (int o = 1; o < 64; o <<= 1) nset += __shfl_xor(nset, o, 64);
        if (lane == 0 && nset && P.replay_count)
            atomicAdd(P.replay_count + kCountSpread + (blockIdx.x & (kCountSpread - 1)), nset);
    }

    // ---- rarest path: the exact Java fold of every coefficient both certificates left open (exact
    //      ties, e.g. k = (0, 2, 2) where the basis products lie in Q(sqrt 2) and the value can be a
    //      rational x.5 exactly: a few per 10^8 coefficients), whole wave, one at a time, written over
    //      the stored value by lane 0.  Its loads wait for the wave's stores (one in-order vmcnt), and
    //      lane 0's store follows its own earlier store of that word (vmcnt(0)), so the exact value is
    //      the one that stays. ----
    if (__builtin_expect(!MEM && __ballot(fm != 0u) != 0ull, 0)) {
        char* rs = wl;  // the wave's region is free again (its last staging round is stored)
        uint32_t n = 0;
        for (;;) {
            const uint64_t who = __ballot(fm != 0u);
            if (who == 0ull) break;
            const int src = (int)__builtin_ctzll(who);
            uint32_t rg, rk;
            e16_flag_pos(fm, src, cube0, rg, rk);
            const int q = replay_fold<8, true>(replay_load<8>(R, rg, rk, lane), rk, lane, (int*)rs,
                                               (double*)(rs + kMaxGroupsDev * 4));
            if (lane == 0) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                P.out[(size_t)rg * CS + rk] = q;
            }
            n++;
            if (lane == src) fm &= fm - 1u;
        }
        if (lane == 0 && P.replay_count) atomicAdd(P.replay_count + (blockIdx.x & (kCountSpread - 1)), n);
    }
}

// DIAGNOSTIC (dct3d_encode_memonly_dev; the output is NOT a DCT): the encode's memory traffic alone --
// the same row loads, the same LDS staging and 1 KiB NT stores of 16 KiB per wave -- with the
// transform, quantisation and certification replaced by a few integer ops on the loaded bytes.  Its
// rate is the ceiling the encode's own traffic reaches on this device (bench.py: ceiling).
template <int D>
__global__ __launch_bounds__(kBlock, 4) void encode_memonly_kernel(EncodeParams P) {
    __shared__ __attribute__((aligned(16))) char lds[kWavesPerBlock * enc_wave_lds<D>()];
    constexpr int NB = (D == 8) ? 8 : 4;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t cube0 = P.g_base + (blockIdx.x * kWavesPerBlock + wave) * kCubesPerWave;
    uint2 raw[D];
    load_rows<D>(P, cube0 + (lane >> 3), cube0 + (lane >> 3) < P.n_cubes, lane & 7, raw);
    if (cube0 >= P.n_cubes) return;
    int32_t qv[8][NB];
#pragma unroll
    for (int ky = 0; ky < 8; ky++)
#pragma unroll
        for (int x = 0; x < NB; x++) qv[ky][x] = (int32_t)((ky & 1 ? raw[x % D].y : raw[x % D].x) >> (ky * 3 % 24)) & 255;
    enc_stage_store<D, true>(P, qv, lds + wave * enc_wave_lds<D>(), lane, cube0);
}

// One wave per uncertified coefficient (flag list), then every coefficient of the whole-cube list.
template <int D>
__global__ __launch_bounds__(256) void encode_fixup_kernel(FixupParams P) {
    constexpr int CS = 64 * D;
    __shared__ int Ssum[4][kMaxGroupsDev];
    __shared__ double prod[4][kMaxGroupsDev];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const ReplayGeom R{P.raster, P.cubes_per_stack, P.nbx, P.width, P.plane, P.stack_stride,
                       P.ngroups, P.coef, P.group_of};
    const uint32_t nf = min(P.counters[0], P.flag_cap);
    const uint32_t ncube = P.counters[1];
    const unsigned long long total = (unsigned long long)nf + (unsigned long long)ncube * CS;
    for (unsigned long long e = (unsigned long long)blockIdx.x * 4 + wave; e < total;
         e += (unsigned long long)gridDim.x * 4) {
        uint32_t g, k;
        if (e < nf) {
            const unsigned long long v = P.flag_list[e];
            g = (uint32_t)(v / CS);
            k = (uint32_t)(v % CS);
        } else {
            const unsigned long long e2 = e - nf;
            g = P.cube_list[e2 / CS];
            k = (uint32_t)(e2 % CS);
        }
        const int q = exact_coef<D>(R, g, k, lane, Ssum[wave], prod[wave]);
        if (lane == 0) P.out[(size_t)g * CS + k] = q;
    }
}

// =============================================================================================
// Fused encode + Exp-Golomb, K1 (dct3d_encode_eg_dev; encoder.c:206-274 up to the deflate)
// =============================================================================================
// The wave's 8 cubes: rows -> transform -> quantise + certify exactly as encode_body, but the
// uncertified coefficients are recorded in a per-lane bit mask (bit ky*NB + x) and replayed by the
// wave itself (exact_coef) after the quantised cubes are staged in LDS as int16 (|q| <= 255*sqrt(cs)
// by Parseval, DC included).  Then lane (c', part) codes stream positions part*VPL .. part*VPL+VPL-1
// of cube c' (diagonal-slice order, CubeUtils.c:5-46; signed order-0 Exp-Golomb, ExpGolomb.c:32-64)
// into its own words of the segment's slot; eg_compact_kernel later concatenates the lanes.
// signed order-0 Exp-Golomb code of the int16 value in the low half of x (ExpGolomb.c:32-64):
// v <= 0 -> 1 - 2v, v > 0 -> 2v; width = 2 * bit_length(code) - 1
__device__ __forceinline__ uint32_t eg_code16(uint32_t x, uint32_t& width) {
    const int32_t v = (int32_t)(int16_t)(uint16_t)x;
    const uint32_t ng = (uint32_t)(-v);
    const uint32_t code = ((ng << 1) ^ (uint32_t)((int32_t)ng >> 31)) + 1u;
    width = 63u - 2u * (uint32_t)__builtin_clz(code);  // code >= 1: a plain v_ffbh_u32 (no zero case)
    return code;
}

// Decoupled look-back (single-pass fused encode): the exclusive stream offset of segment s from the
// look-back words of segments < s -- kLbK x 64 at a time, kLbK independent loads per lane (sc1 loads:
// agent-scope atomics), so that a walk past the segments still in flight (thousands) takes a few
// round trips.  A window counts once every segment up to the nearest inclusive prefix has at least its
// aggregate; the wave re-polls otherwise.  Segments are dispatched in order and publish their aggregate
// before they look back, so the wait is short; a bounded spin gives up (returns false) instead of hanging.
constexpr uint64_t kLbP = 1ull << 63, kLbA = 1ull << 62, kLbVal = kLbA - 1;
constexpr int kLbK = 1;
__device__ __forceinline__ uint64_t lanes_upto(int fp, int k) {  // lanes l with 64k + l <= fp
    const int r = fp - 64 * k;
    return r < 0 ? 0ull : (r >= 63 ? ~0ull : ((2ull << r) - 1ull));
}
__device__ __forceinline__ bool lookback_offset(const uint64_t* st, uint64_t s, uint64_t carry, int lane,
                                                uint64_t& excl) {
    excl = 0;
    int64_t j0 = (int64_t)s - 1;
    for (uint32_t spins = 0; spins < (1u << 20);) {
        uint64_t v[kLbK];
#pragma unroll
        for (int k = 0; k < kLbK; k++) {
            const int64_t j = j0 - lane - 64 * k;
            v[k] = j >= 0 ? __hip_atomic_load(&st[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                          : (kLbP | carry);  // before segment 0: the carried bits
        }
        int fp = 64 * kLbK;  // window index (64k + lane) of the nearest inclusive prefix
#pragma unroll
        for (int k = kLbK - 1; k >= 0; k--) {
            const uint64_t pm = __ballot((v[k] & kLbP) != 0);
            if (pm) fp = 64 * k + __builtin_ctzll(pm);
        }
        bool gave_up = false, missing = false;
        uint64_t c = 0;
#pragma unroll
        for (int k = 0; k < kLbK; k++) {
            const uint64_t need = lanes_upto(fp, k);
            gave_up |= (__ballot((v[k] & (kLbP | kLbA)) == (kLbP | kLbA)) & need) != 0;
            missing |= (__ballot((v[k] & (kLbP | kLbA)) == 0) & need) != 0;
            c += ((need >> lane) & 1) ? (v[k] & kLbVal) : 0ull;
        }
        if (gave_up) return false;
        if (missing) {  // not published yet: poll again
            spins++;
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
        excl += c;
        if (fp < 64 * kLbK) return true;
        j0 -= 64 * kLbK;
    }
    return false;
}

template <int D, bool SP>
__global__ __launch_bounds__(kBlock, 4) void encode_eg_kernel(EncodeParams P, EgFusedParams E) {
    constexpr int CS = 64 * D;
    constexpr int NB = (D == 8) ? 8 : 4;
    constexpr int NI = 7 + NB;
    constexpr int VPL = CS / 8;            // stream values per lane
    constexpr int CUBE_B = 2 * CS + 16;    // int16 cube-major staging per cube (+16 B: bank spread)
    static_assert(8 * CUBE_B <= enc_wave_lds<D>(), "int16 staging must fit the wave region");
    __shared__ __attribute__((aligned(16))) char lds[kWavesPerBlock * enc_wave_lds<D>()];
    // exact-replay scratch (kMaxGroupsDev sums + products per wave): 8x8x8 keeps it in the tail of the
    // wave's region behind the int16 staging, so that the block fits a quarter of the CU's LDS together
    // with the table copy; 8x8x4's region has no such room
    constexpr int RS_B = kMaxGroupsDev * (4 + 8);
    constexpr bool RS_TAIL = 8 * CUBE_B + RS_B <= enc_wave_lds<D>();
    __shared__ __attribute__((aligned(16))) char rs_extra[RS_TAIL ? 16 : kWavesPerBlock * RS_B];
    __shared__ __attribute__((aligned(16))) uint16_t s_pos[CS];  // stream position -> byte offset in a cube
    __shared__ float4 s_tab[kTabN];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t wid = blockIdx.x * kWavesPerBlock + wave;  // segment index
    const uint32_t cube0 = wid * kCubesPerWave;
    uint2 raw[D];
    load_rows<D>(P, cube0 + (lane >> 3), cube0 + (lane >> 3) < P.n_cubes, lane & 7, raw);  // in flight first
    {  // both loads in flight before the LDS writes (a strided loop waited one round trip per pass)
        static_assert(CS % kBlock == 0, "whole passes");
        uint16_t t[CS / kBlock];
#pragma unroll
        for (int r = 0; r < CS / kBlock; r++) t[r] = E.diag[threadIdx.x + r * kBlock];
#pragma unroll
        for (int r = 0; r < CS / kBlock; r++) s_pos[threadIdx.x + r * kBlock] = (uint16_t)(2 * t[r]);
    }
    __syncthreads();
    if (cube0 >= P.n_cubes) return;  // wave-uniform, after the barrier
    enc_tables(P, s_tab, lane);
    char* wl = lds + wave * enc_wave_lds<D>();
    char* rs = RS_TAIL ? wl + 8 * CUBE_B : rs_extra + wave * RS_B;
    static_assert((8 * CUBE_B) % 8 == 0 && RS_B % 8 == 0, "replay scratch alignment");
    const int c = lane >> 3, j = lane & 7;
    const int kz = (D == 8) ? j : (j >> 1);
    const int kx0 = (D == 8) ? 0 : (j & 1) * 4;
    const int so = kz + kx0;
    const bool valid = cube0 + c < P.n_cubes;

    float a[D][8];
    to_float<D>(raw, a);
    uint32_t S;
    int m;
    float A;
    cube_stats<D>(raw, a, S, m, A);
    asm volatile("" : "+v"(S), "+v"(m), "+v"(A));
    float b[8][NB];
    forward_cube<D, NB>(a, m, c, j, wl, b);

    int sz = so;
    float rr[NI], thr[NI];
    int32_t qv[8][NB];
    uint32_t fm_lo = 0, fm_hi = 0;  // uncertified mask: bit ky*NB + x (64 bits for NB = 8)
#pragma unroll
    for (int ky = 0; ky < 8; ky++) {
        pin(b[ky]);
        tab_window<NB, NI>(s_tab, sz, ky, A, rr, thr);
        bool f = false;
        float qq[NB];
#pragma unroll
        for (int x = 0; x < NB; x++) {
            qq[x] = b[ky][x] * rr[ky + x];
            const float n = __builtin_rintf(qq[x]);
            f |= __builtin_fabsf(qq[x] - n) >= thr[ky + x];
            qv[ky][x] = (int32_t)n;
        }
        if (__builtin_expect(f, 0)) {
            uint32_t bits = 0;
#pragma unroll
            for (int x = 0; x < NB; x++)
                if (__builtin_fabsf(qq[x] - __builtin_rintf(qq[x])) >= thr[ky + x]) bits |= 1u << x;
            const int sh = ky * NB;
            if (sh < 32) fm_lo |= bits << sh;
            else fm_hi |= bits << (sh - 32);
        }
        pin(qv[ky]);
        asm volatile("" : "+v"(fm_lo), "+v"(fm_hi));
    }
    if (j == 0) {
        qv[0][0] = java_round_dev((double)S * P.coef_dc);  // exact DC (single Java group)
        fm_lo &= ~1u;
    }
    if (!valid) fm_lo = fm_hi = 0;

    // stage the cubes as int16, cube-major (k = (kz*8 + ky)*8 + kx at byte 2k of cube c)
#pragma unroll
    for (int ky = 0; ky < 8; ky++) {
        char* row = wl + c * CUBE_B + 2 * ((kz * 8 + ky) * 8 + kx0);
        if constexpr (D == 8) {
            *(uint4*)row = make_uint4(__builtin_amdgcn_perm(qv[ky][1], qv[ky][0], 0x05040100u),
                                      __builtin_amdgcn_perm(qv[ky][3], qv[ky][2], 0x05040100u),
                                      __builtin_amdgcn_perm(qv[ky][5], qv[ky][4], 0x05040100u),
                                      __builtin_amdgcn_perm(qv[ky][7], qv[ky][6], 0x05040100u));
        } else {
            *(uint2*)row = make_uint2(__builtin_amdgcn_perm(qv[ky][1], qv[ky][0], 0x05040100u),
                                      __builtin_amdgcn_perm(qv[ky][3], qv[ky][2], 0x05040100u));
        }
    }
    wave_lds_sync();

    // exact replay of the uncertified coefficients, one at a time by the whole wave (rare)
    {
        const ReplayGeom R{P.raster, P.cubes_per_stack, P.nbx, P.width, P.plane, P.stack_stride,
                           E.ngroups, E.coef, E.group_of};
        for (;;) {
            const unsigned long long who = __ballot((fm_lo | fm_hi) != 0u);
            if (who == 0ull) break;
            const int src = __builtin_ctzll(who);
            const int mybit = fm_lo ? __builtin_ctz(fm_lo) : (fm_hi ? 32 + __builtin_ctz(fm_hi) : 0);
            const int bit = __shfl(mybit, src, 64);
            const int sj = src & 7, sc = src >> 3;
            const int skz = (D == 8) ? sj : (sj >> 1), skx0 = (D == 8) ? 0 : (sj & 1) * 4;
            const uint32_t k = (uint32_t)((skz * 8 + bit / NB) * 8 + skx0 + bit % NB);
            const int q = exact_coef<D>(R, cube0 + sc, k, lane, (int*)rs, (double*)(rs + kMaxGroupsDev * 4));
            if (lane == 0) *(int16_t*)(wl + sc * CUBE_B + 2 * k) = (int16_t)q;
            if (lane == src) {
                if (fm_lo) fm_lo &= fm_lo - 1;
                else fm_hi &= fm_hi - 1;
            }
            wave_lds_sync();
        }
    }

    // Exp-Golomb: lane (cp, part) codes stream positions part*VPL .. +VPL-1 of cube cp, read from the
    // staged cube, with a 64-bit accumulator: one MSB-first word out whenever 32 bits are pending
    // (width <= 27, + 31 pending), word i of lane l at slot row i (i*64 + l).  eg_compact_kernel
    // concatenates the lanes.  (Buffering the words in LDS first needs the values in registers to
    // free the region: +6 % kernel time for the pack / unpack, more than the scattered stores cost.)
    const int cp = lane >> 3, part = lane & 7;
    const bool lvalid = cube0 + cp < P.n_cubes;
    const char* cb = wl + cp * CUBE_B;
    if constexpr (SP) {
        // ---- single pass: lane bit counts, segment offset by look-back, words straight into place ----
        uint32_t lb = 0;
        if (lvalid) {
#pragma unroll 1
            for (int i0 = 0; i0 < VPL; i0 += 8) {
                const uint4 pp = *(const uint4*)&s_pos[part * VPL + i0];
                const uint32_t pw[4] = {pp.x, pp.y, pp.z, pp.w};
#pragma unroll
                for (int e = 0; e < 8; e++) {
                    uint32_t width;
                    (void)eg_code16(*(const uint16_t*)(cb + ((pw[e >> 1] >> (16 * (e & 1))) & 0xFFFFu)), width);
                    lb += width;
                }
            }
        }
        uint32_t incl = lb;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t t = __shfl_up(incl, o, 64);
            if (lane >= o) incl += t;
        }
        const uint32_t tot = __shfl(incl, 63, 64);
        const uint64_t s = wid;
        if (lane == 0) __hip_atomic_store(&E.seg_state[s], kLbA | tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        uint64_t base = 0;
        const bool ok = lookback_offset(E.seg_state, s, E.carry_bits, lane, base);
        if (lane == 0)
            __hip_atomic_store(&E.seg_state[s], ok ? (kLbP | (base + tot)) : (kLbP | kLbA), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        if (!ok) {  // the host re-runs the call with the two-pass path
            if (lane == 0) atomicOr((unsigned int*)&E.status[1], 4u);
            return;
        }
        if (lane == 0) {
            E.seg_off[s] = base;
            E.seg_bits[s] = tot;
            if (cube0 + kCubesPerWave >= P.n_cubes) E.status[0] = base + tot;  // the last segment: total
        }
        if ((base + tot + 31) / 32 > E.out_cap_words) {  // wave-uniform; nothing is written past the end
            if (lane == 0) atomicOr((unsigned int*)&E.status[1], 1u);
            return;
        }
        // eg_compact_kernel's placement, fed word by word from the coder instead of from a slot
        const uint64_t start = base + (incl - lb);
        const uint32_t r = (uint32_t)(start & 31);
        uint32_t* const outw = E.out + (start >> 5);
        const uint32_t ndst = lb ? (uint32_t)(((start + lb - 1) >> 5) - (start >> 5) + 1) : 0u;
        uint32_t prev = 0, first = 0, last = 0, d = 0;
        auto put = [&](uint32_t cur) {
            const uint32_t v = r ? ((cur >> r) | (prev << (32 - r))) : cur;
            prev = cur;
            if (d == 0) first = v;
            if (d == ndst - 1) last = v;
            if (d != 0 && d != ndst - 1) outw[d] = __builtin_bswap32(v);
            d++;
        };
        uint64_t acc = 0;
        uint32_t nb = 0;
        if (lvalid) {
#pragma unroll 1
            for (int i0 = 0; i0 < VPL; i0 += 8) {
                const uint4 pp = *(const uint4*)&s_pos[part * VPL + i0];
                const uint32_t pw[4] = {pp.x, pp.y, pp.z, pp.w};
                uint32_t v[8];
#pragma unroll
                for (int e = 0; e < 8; e++) v[e] = *(const uint16_t*)(cb + ((pw[e >> 1] >> (16 * (e & 1))) & 0xFFFFu));
#pragma unroll
                for (int e = 0; e < 8; e++) {
                    uint32_t width;
                    const uint32_t code = eg_code16(v[e], width);
                    acc = (acc << width) | code;
                    nb += width;
                    if (nb >= 32u) {
                        nb -= 32u;
                        put((uint32_t)(acc >> nb));
                    }
                }
            }
            if (nb) put((uint32_t)(acc << (32u - nb)));
            if (d < ndst) put(0u);  // the last word holds only the shifted-out bits of the previous one
        }
        const uint32_t nlb = __shfl_down(lb, 1, 64);
        const bool next_shares = lane < 63 && nlb != 0u && ((start + lb) & 31) != 0;
        const bool last_lane = lb != 0u && (lane == 63 || nlb == 0u);
        const uint32_t nfirst = __shfl_down(first, 1, 64);
        if (next_shares) last |= nfirst;
        if (ndst == 0) return;
        const bool shares_prev = lane > 0 && r != 0;
        if (ndst == 1) {
            if (lane == 0) E.head[s] = __builtin_bswap32(first);
            else if (last_lane) E.tail[s] = __builtin_bswap32(last);
            else outw[0] = __builtin_bswap32(last);
            return;
        }
        if (lane == 0) E.head[s] = __builtin_bswap32(first);
        else if (!shares_prev) outw[0] = __builtin_bswap32(first);
        if (last_lane) E.tail[s] = __builtin_bswap32(last);
        else outw[ndst - 1] = __builtin_bswap32(last);
        return;
    }
    // the segment's slot base is wave-uniform (scalar); each store adds a 32-bit lane offset
    char* const seg = (char*)(E.slot + (size_t)__builtin_amdgcn_readfirstlane(wid) * E.seg_cap);
    uint32_t dofs = (uint32_t)lane * 4u;  // byte offset of the lane's next word: (nw * 64 + lane) * 4
    uint64_t acc = 0;
    uint32_t nb = 0;
    if (lvalid) {
#pragma unroll 1
        for (int i0 = 0; i0 < VPL; i0 += 8) {
            const uint4 pp = *(const uint4*)&s_pos[part * VPL + i0];
            const uint32_t pw[4] = {pp.x, pp.y, pp.z, pp.w};
            uint32_t v[8];
#pragma unroll
            for (int e = 0; e < 8; e++) v[e] = *(const uint16_t*)(cb + ((pw[e >> 1] >> (16 * (e & 1))) & 0xFFFFu));
#pragma unroll
            for (int e = 0; e < 8; e++) {
                uint32_t width;
                const uint32_t code = eg_code16(v[e], width);
                acc = (acc << width) | code;
                nb += width;
                if (nb >= 32u) {
                    nb -= 32u;
                    *(uint32_t*)(seg + dofs) = (uint32_t)(acc >> nb);
                    dofs += 256u;
                }
            }
        }
        if (nb) *(uint32_t*)(seg + dofs) = (uint32_t)(acc << (32u - nb));
    }
    const uint32_t nw = (dofs - (uint32_t)lane * 4u) >> 8;  // full words stored
    const uint32_t lbits = lvalid ? nw * 32u + nb : 0u;
    E.lane_bits[(size_t)wid * 64 + lane] = (uint16_t)lbits;
    uint32_t tot = lbits;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o, 64);
    if (lane == 0) E.seg_bits[wid] = tot;
}


// =============================================================================================
// Fused decode (fp64, certified)
// =============================================================================================
// ---------------------------------------------------------------------------------------------
// Decode v1: 2*D lanes per cube, 32 doubles per lane (<= 128 VGPRs, 4 waves per SIMD).
//   lane = c2*32 + h*16 + c1*D + k   (cube c = c2*(CPW/2) + c1; h = bit 4; k = low bits)
//   layout A (pass Y): lane (c, kz=k, h) holds b[ky][e], kx = 4h + e        (lines along ky)
//   layout B (pass X): lane (c, kz=k, h) holds a[r][x],  y  = 4h + r        (lines along kx)
//   layout C (pass Z): D=8: lane (c, y=k, h) holds cz[z][e], x = 4h + e      (lines along z)
//                      D=4: lane (c, y=4h+k)  holds cz[z][x]
//   A -> B is a lane-pair exchange (lanes l, l^16) by v_permlane16_swap: no LDS.
//   B -> C goes through the wave's LDS region in two rounds (D=8: z halves, D=4: x halves), 8 KiB each.
// Inputs are staged through the same region (1 KiB per load instruction).  The per-axis operation
// sequence (dequantise, idct8/4 along Y, X, Z) is the one the planner's fp64 analysis bounds.
// Certify + clamp: with m = amax*G + E (+2^-43 for the two roundings below, |v| < 1024),
//   lo = v - m, hi = v + m;  out = min(cvt_u32(lo), 255)  unless cvt_u32(lo) != cvt_u32(hi).
// cvt_u32 (v_cvt_u32_f64) truncates and saturates (negative -> 0), so min(cvt_u32(x), 255) is the
// monotone map x -> (byte) clamp(x, 0, 255) of InverseDCT.java:74-80 / Decoder.java:112, and equal
// values at lo and hi prove the Java value (within [lo, hi]) maps to the same byte.
// ---------------------------------------------------------------------------------------------
constexpr int kDecWaveLds = 9216;

template <int D>
struct DecGeom {
    static constexpr int CS = 64 * D;
    static constexpr int LPC = 2 * D;          // lanes per cube
    static constexpr int CPW = 64 / LPC;       // cubes per wave: 4 (D=8) | 8 (D=4)
    static constexpr int SA_F = 288;           // staging face stride (256 B + 32 B pad)
    static constexpr int SA_C = D * SA_F;      // staging cube stride
    // B->C round strides (bank-conflict-free for D=8 by the guide's lane-group rules; D=4 best found)
    static constexpr int TZ = (D == 8) ? 528 : 256;    // z stride (D=8: 8 rows x 64 B + 16)
    static constexpr int TC = (D == 8) ? 2128 : 1040;  // cube stride
    static_assert(CPW * SA_C <= kDecWaveLds && CPW * TC <= kDecWaveLds, "wave LDS region");
    // slot of row y in face z (D=4 swizzles rows by z: bank spread of the 8-lane-per-cube reads)
    static __device__ __forceinline__ int tslot(int z, int y) { return (D == 8) ? y : (y ^ z); }
};

__device__ __forceinline__ void swap16(double& a, double& b) {
    const uint64_t ua = __builtin_bit_cast(uint64_t, a), ub = __builtin_bit_cast(uint64_t, b);
    const auto lo = __builtin_amdgcn_permlane16_swap((uint32_t)ua, (uint32_t)ub, false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap((uint32_t)(ua >> 32), (uint32_t)(ub >> 32), false, false);
    a = __builtin_bit_cast(double, ((uint64_t)hi[0] << 32) | lo[0]);
    b = __builtin_bit_cast(double, ((uint64_t)hi[1] << 32) | lo[1]);
}

__device__ __forceinline__ uint32_t cvt_u32_sat(double v) {
    uint32_t t;
    asm("v_cvt_u32_f64 %0, %1" : "=v"(t) : "v"(v));
    return t;
}

// Fixed-point view of a decoded value, for the decode's certificate (decode_tile): with |v| < 2^19,
// w = v + 1.5 * 2^20 lies in [2^20, 2^21), whose ulp is 2^-32, so one fp64 add (rounding error
// <= 2^-33) leaves frac(v) * 2^32 in w's low word and 0x41380000 + floor(v) in its high word
// (0x413: the biased exponent of 2^20; 2^19: the offset 0.5 * 2^20).
constexpr double kFixMagic = 1572864.0;  // 1.5 * 2^20
constexpr uint32_t kFixHi = 0x41380000u;
// max(0, hi - kFixHi): max(0, floor(v)) in one VALU op (unsigned subtract, clamped at 0)
__device__ __forceinline__ uint32_t fix_floor0(uint32_t hi) {
    uint32_t t;
    asm("v_sub_u32_e64 %0, %1, %2 clamp" : "=v"(t) : "v"(hi), "s"(kFixHi));
    return t;
}

// staged input of one tile (CPW cubes, 8 KiB): 8 coalesced 1 KiB loads per wave
// (4-byte values: int32 quantised cubes, or the float cubes of the drop-in kernels)
template <int D>
__device__ __forceinline__ void dec_load_tile_p(const char* in, uint32_t n_cubes, uint32_t cube0, int lane,
                                                int4 (&v)[8]) {
    using G = DecGeom<D>;
    const char* inb = in + (size_t)cube0 * G::CS * 4;
    if (cube0 + G::CPW <= n_cubes) {  // wave-uniform: every cube of the tile exists
#pragma unroll
        for (int t = 0; t < 8; t++) {
            const i32x4_t x = __builtin_nontemporal_load((const i32x4_t*)(inb + (size_t)(t * 64 + lane) * 16));
            v[t] = make_int4(x.x, x.y, x.z, x.w);
        }
    } else {
#pragma unroll
        for (int t = 0; t < 8; t++) {
            const int q = t * 64 + lane;
            v[t] = make_int4(0, 0, 0, 0);
            if (cube0 + q / (G::CS / 4) < n_cubes) v[t] = *(const int4*)(inb + (size_t)q * 16);
        }
    }
}
template <int D>
__device__ __forceinline__ void dec_load_tile(const DecodeParams& P, uint32_t cube0, int lane, int4 (&v)[8]) {
    dec_load_tile_p<D>((const char*)P.in, P.n_cubes, cube0, lane, v);
}
template <int D>
__device__ __forceinline__ void dec_stage_tile(char* wl, int lane, const int4 (&v)[8]) {
    using G = DecGeom<D>;
#pragma unroll
    for (int t = 0; t < 8; t++) {
        const int q = t * 64 + lane;
        *(int4*)(wl + (q / (G::CS / 4)) * G::SA_C + ((q >> 4) % D) * G::SA_F + (q & 15) * 16) = v[t];
    }
}

// ---- B -> C through LDS in two rounds (D=8: z halves, D=4: x halves); every lane reads in
//      every round into fixed registers (no lane-divergent definitions to merge) ----
//   in:  layout B, lane (c, kz=k, h): row r (y = 4h + r): x 0..3 in b[r][.], x 4..7 in b[4 + r][.]
//   out: layout C, D=8: lane (c, y=k, h) cz[z][e] (x = 4h + e); D=4: lane (c, y=4h+k) cz[z][x]
template <int D>
__device__ __forceinline__ void dec_b_to_c(const double (&b)[8][4], double (&cz)[D][(D == 8) ? 4 : 8], char* wl,
                                           int c, int k, int h) {
    using G = DecGeom<D>;
#pragma unroll
    for (int rd = 0; rd < 2; rd++) {
        wave_lds_sync();
        if constexpr (D == 8) {
            if ((k >> 2) == rd) {  // writers: this round's z half; rows of 8 x (64 B)
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    char* dst = wl + c * G::TC + (k & 3) * G::TZ + (4 * h + r) * 64;
                    *(double2*)(dst) = make_double2(b[r][0], b[r][1]);
                    *(double2*)(dst + 16) = make_double2(b[r][2], b[r][3]);
                    *(double2*)(dst + 32) = make_double2(b[4 + r][0], b[4 + r][1]);
                    *(double2*)(dst + 48) = make_double2(b[4 + r][2], b[4 + r][3]);
                }
            }
            wave_lds_sync();
#pragma unroll
            for (int zr = 0; zr < 4; zr++) {
                const char* src = wl + c * G::TC + zr * G::TZ + k * 64 + h * 32;
                const double2 t0 = *(const double2*)(src), t1 = *(const double2*)(src + 16);
                cz[4 * rd + zr][0] = t0.x; cz[4 * rd + zr][1] = t0.y;
                cz[4 * rd + zr][2] = t1.x; cz[4 * rd + zr][3] = t1.y;
            }
        } else {
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const double* sv = (rd == 0) ? b[r] : b[4 + r];
                char* dst = wl + c * G::TC + k * G::TZ + G::tslot(k, 4 * h + r) * 32;
                *(double2*)(dst) = make_double2(sv[0], sv[1]);
                *(double2*)(dst + 16) = make_double2(sv[2], sv[3]);
            }
            wave_lds_sync();
            const int y = 4 * h + k;
#pragma unroll
            for (int z = 0; z < 4; z++) {
                const char* src = wl + c * G::TC + z * G::TZ + G::tslot(z, y) * 32;
                const double2 t0 = *(const double2*)(src), t1 = *(const double2*)(src + 16);
                cz[z][4 * rd + 0] = t0.x; cz[z][4 * rd + 1] = t0.y;
                cz[z][4 * rd + 2] = t1.x; cz[z][4 * rd + 3] = t1.y;
            }
        }
    }
}

// One tile (CPW cubes) from the staged input in the wave's LDS region to the raster.  after_a() runs
// once the staged input is in registers (the persistent variant issues the next tile's loads there).
// PG: butterflies per pin group (1: one at a time, 2 / 4: that many interleaved, 0: no pins)
template <int D, int PG, class AfterA>
__device__ __forceinline__ void decode_tile(const DecodeParams& P, char* wl, int lane, uint32_t cube0,
                                            AfterA&& after_a) {
    using G = DecGeom<D>;
    constexpr int CPW = G::CPW;
    constexpr int NXC = (D == 8) ? 4 : 8;  // x values per lane in layout C
    const int h = (lane >> 4) & 1;
    const int k = lane & (D - 1);
    const int c = (lane >> 5) * (CPW / 2) + ((lane & 15) / D);
    const uint32_t g = cube0 + c;
    const bool valid = g < P.n_cubes;

    // ---- layout A: dequantise, amax ----
    // cf = q * step exactly: a 24-bit integer multiply (|q| < 2^23 checked; |q * step| < 2^30), then
    // an exact conversion to fp64.  Out-of-range q (never produced by the encoder) sends the cube to
    // the exact replay.  amax = max |q * step| from integer max / min.
    double b[8][4];
    float amax_f;
    bool q_range_bad;
    {
        const int sb = 5 * (4 * h + k);                     // step = sb + 5 (e + ky); DC (e = ky = 0): 1
        int stp[11];
        stp[0] = max(sb, 1);
#pragma unroll
        for (int j = 1; j < 11; j++) stp[j] = sb + 5 * j;
        const char* src = wl + c * G::SA_C + k * G::SA_F + h * 16;
        int4 raw[8];  // all eight LDS reads in flight before the first use
#pragma unroll
        for (int ky = 0; ky < 8; ky++) raw[ky] = *(const int4*)(src + ky * 32);
        int qmax = INT32_MIN, qmin = INT32_MAX, tmax = 0, tmin = 0;
#pragma unroll
        for (int ky = 0; ky < 8; ky++) {
            const int vv[4] = {raw[ky].x, raw[ky].y, raw[ky].z, raw[ky].w};
            int t[4];
#pragma unroll
            for (int e = 0; e < 4; e++) {
                t[e] = __mul24(vv[e], stp[e + ky]);
                b[ky][e] = (double)t[e];
            }
            qmax = max(qmax, max(max(vv[0], vv[1]), max(vv[2], vv[3])));
            qmin = min(qmin, min(min(vv[0], vv[1]), min(vv[2], vv[3])));
            tmax = max(tmax, max(max(t[0], t[1]), max(t[2], t[3])));
            tmin = min(tmin, min(min(t[0], t[1]), min(t[2], t[3])));
        }
        q_range_bad = (qmax > 0x7FFFFF) | (qmin < -0x800000);
        // float upper bound of amax (nearest rounding is within 2^-24 relative; the product with
        // 1 + 2^-22 rounds to at least amax): the cube reduction then moves one dword per step
        amax_f = (float)max(tmax, -tmin) * (1.0f + 0x1p-22f);
    }
    after_a();
    // amax over the cube's lanes (k bits, then bit 4): DPP within the row, one permlane16 swap across
    amax_f = fmaxf(amax_f, __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, amax_f), 0xB1, 0xF, 0xF, false)));  // quad_perm xor 1
    amax_f = fmaxf(amax_f, __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, amax_f), 0x4E, 0xF, 0xF, false)));  // quad_perm xor 2
    if constexpr (D == 8)
        amax_f = fmaxf(amax_f, __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, amax_f), 0x141, 0xF, 0xF, false)));  // row_half_mirror
    {
        const auto sw = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(uint32_t, amax_f), __builtin_bit_cast(uint32_t, amax_f), false, false);
        amax_f = fmaxf(__builtin_bit_cast(float, (uint32_t)sw[0]), __builtin_bit_cast(float, (uint32_t)sw[1]));
    }
    const double amax = (double)amax_f;

    // ---- inverse pass Y ----
    constexpr int G1 = PG == 0 ? 4 : PG;
#pragma unroll
    for (int e0 = 0; e0 < 4; e0 += G1) {
        double col[G1][8];
#pragma unroll
        for (int i = 0; i < G1; i++)
#pragma unroll
            for (int y = 0; y < 8; y++) col[i][y] = b[y][e0 + i];
        if (PG) for (int i = 0; i < G1; i++) pin(col[i]);
#pragma unroll
        for (int i = 0; i < G1; i++) idct8(col[i]);
        if (PG) for (int i = 0; i < G1; i++) pin(col[i]);
#pragma unroll
        for (int i = 0; i < G1; i++)
#pragma unroll
            for (int y = 0; y < 8; y++) b[y][e0 + i] = col[i][y];
    }

    // ---- A -> B: swap the off-diagonal 4x4 blocks of the lane pair (l, l^16) ----
#pragma unroll
    for (int r = 0; r < 4; r++)
#pragma unroll
        for (int e = 0; e < 4; e++) swap16(b[r][e], b[4 + r][e]);
    // now row r of this lane (y = 4h + r): x 0..3 in b[r][.], x 4..7 in b[4 + r][.]

    // ---- inverse pass X ----
#pragma unroll
    for (int r0 = 0; r0 < 4; r0 += G1) {
        double row[G1][8];
#pragma unroll
        for (int i = 0; i < G1; i++)
#pragma unroll
            for (int e = 0; e < 4; e++) {
                row[i][e] = b[r0 + i][e];
                row[i][4 + e] = b[4 + r0 + i][e];
            }
        if (PG) for (int i = 0; i < G1; i++) pin(row[i]);
#pragma unroll
        for (int i = 0; i < G1; i++) idct8(row[i]);
        if (PG) for (int i = 0; i < G1; i++) pin(row[i]);
#pragma unroll
        for (int i = 0; i < G1; i++)
#pragma unroll
            for (int e = 0; e < 4; e++) {
                b[r0 + i][e] = row[i][e];
                b[4 + r0 + i][e] = row[i][4 + e];
            }
    }

    double cz[D][NXC];
    dec_b_to_c<D>(b, cz, wl, c, k, h);

    // ---- inverse pass Z ----
    constexpr int G3 = PG == 0 ? NXC : PG;
#pragma unroll
    for (int e0 = 0; e0 < NXC; e0 += G3) {
        double col[G3][D];
#pragma unroll
        for (int i = 0; i < G3; i++)
#pragma unroll
            for (int z = 0; z < D; z++) col[i][z] = cz[z][e0 + i];
        if (PG) for (int i = 0; i < G3; i++) pin(col[i]);
#pragma unroll
        for (int i = 0; i < G3; i++) idctN<D>(col[i]);
        if (PG) for (int i = 0; i < G3; i++) pin(col[i]);
#pragma unroll
        for (int i = 0; i < G3; i++)
#pragma unroll
            for (int z = 0; z < D; z++) cz[z][e0 + i] = col[i][z];
    }

    // ---- certify, clamp + truncate, store ----
    // |v - v_java| <= m (dct3d_plan.cpp).  The byte is min(max(0, floor(v)), 255), monotone in v, so it
    // is Java's byte when floor is constant over [v - m, v + m]: frac(v) >= m and frac(v) + m < 1.  In
    // the fixed-point view (kFixMagic) lo = frac(v) 2^32 to within 1/2 unit, so with
    // mi = m 2^32 + 1/2 rounded up, lo in [mi, 2^32 - 1 - mi] proves it: (lo - mi) <= 2^32 - 1 - 2 mi
    // as unsigned.  |v| < 2^19 holds when amax < 2^14: |v| <= amax * sum_k |c(n, k)| <= amax 8^1.5;
    // a larger amax (never from an encoder of 8-bit frames) sends the cube to the replay.
    const double m = amax * P.dec_G + P.dec_E;
    const uint32_t mi = (uint32_t)__builtin_ceil(__fma_rn(m, 0x1p32, 0.5)) + 1u;  // + 1: m's own rounding
    const uint32_t cert_lim = 0xFFFFFFFFu - 2u * mi;
    const int y = (D == 8) ? k : (4 * h + k);
    const int x0 = (D == 8) ? 4 * h : 0;
    bool flag = q_range_bad | (amax_f >= 16384.0f);
    uint32_t outw[D][NXC / 4];
    const uint32_t c255 = 255u;
#pragma unroll
    for (int z = 0; z < D; z++) {
#pragma unroll
        for (int wd = 0; wd < NXC / 4; wd++) {
            uint32_t w = 0;
#pragma unroll
            for (int e = 0; e < 4; e++) {
                const uint64_t fx = __builtin_bit_cast(uint64_t, __dadd_rn(cz[z][4 * wd + e], kFixMagic));
                const uint32_t tl = fix_floor0((uint32_t)(fx >> 32));
                flag |= ((uint32_t)fx - mi) > cert_lim;
                // byte e of w = min(tl, 255) (SDWA byte insert: the other bytes are preserved)
                if (e == 0) w = min(tl, 255u);
                else if (e == 1) asm("v_min_u32_sdwa %0, %1, %2 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD" : "+v"(w) : "v"(tl), "v"(c255));
                else if (e == 2) asm("v_min_u32_sdwa %0, %1, %2 dst_sel:BYTE_2 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD" : "+v"(w) : "v"(tl), "v"(c255));
                else asm("v_min_u32_sdwa %0, %1, %2 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD" : "+v"(w) : "v"(tl), "v"(c255));
            }
            asm volatile("" : "+v"(w));  // one output word at a time (bounded live range)
            outw[z][wd] = w;
        }
    }
    if (valid) {
        const uint32_t s = fdiv(g, P.div_cps);
        const uint32_t rr = g - s * P.cubes_per_stack;
        const uint32_t by = fdiv(rr, P.div_nbx), bx = rr - by * P.nbx;
        uint8_t* dst = P.out + (size_t)s * P.stack_stride + (size_t)(by * 8 + y) * P.width + bx * 8 + x0;
#pragma unroll
        for (int z = 0; z < D; z++) {
            if constexpr (NXC == 4) *(uint32_t*)(dst + (size_t)z * P.plane) = outw[z][0];
            else *(uint2*)(dst + (size_t)z * P.plane) = make_uint2(outw[z][0], outw[z][1]);
        }
    }
    // uncertified pixels are rare (tens per 2e9): the cube goes to the whole-cube replay list (one
    // lane per cube appends it), which keeps the main path free of per-pixel bookkeeping
    const unsigned long long fl = __ballot(flag && valid);
    if (__builtin_expect(fl != 0ull, 0)) {
        const int base = (lane & 32) + ((lane & 15) & ~(D - 1));
        const unsigned long long cmask = ((unsigned long long)((1u << D) - 1) << base) |
                                         ((unsigned long long)((1u << D) - 1) << (base + 16));
        if ((fl & cmask) != 0ull && (int)__builtin_ctzll(fl & cmask) == lane) {
            const uint32_t idx = atomicAdd(&P.counters[1], 1u);
            P.cube_list[idx] = g;
        }
    }
}

template <int D, int PG>
__global__ __launch_bounds__(kBlock, 4) void decode_kernel(DecodeParams P) {
    __shared__ __attribute__((aligned(16))) char lds[kWavesPerBlock * kDecWaveLds];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    char* wl = lds + wave * kDecWaveLds;
    const uint32_t cube0 = (blockIdx.x * kWavesPerBlock + wave) * DecGeom<D>::CPW;
    int4 v[8];
    dec_load_tile<D>(P, cube0, lane, v);
    dec_stage_tile<D>(wl, lane, v);
    wave_lds_sync();
    decode_tile<D, PG>(P, wl, lane, cube0, [] {});
}

// =============================================================================================
// Drop-in (A): float cube-major -> float cube-major, fp64 internal (3dDCT.cl:43-143 / 164-265)
// =============================================================================================
// The decode kernel's geometry (2*D lanes per cube, 32 doubles per lane, staged 1 KiB loads, the
// lane-pair swap and the two LDS rounds), with the forward (DCT-II) or inverse (DCT-III, clamped to
// [0,255] as 3dDCT.cl:257-261) butterflies along Y, X, Z.  Layout C stores f32 cube-major directly:
// for D = 8 a store instruction covers one 256-byte z face of each of the wave's 4 cubes.
template <bool INV>
__device__ __forceinline__ void f64_line8(double (&x)[8]) {
    if constexpr (INV) idct8(x);
    else fdct8<false, false>(x, 0.0);
}
template <int D, bool INV>
__global__ __launch_bounds__(kBlock, 4) void cube_f32_kernel(const float* __restrict__ in, float* __restrict__ out,
                                                             uint32_t n_cubes) {
    using G = DecGeom<D>;
    constexpr int CPW = G::CPW;
    constexpr int NXC = (D == 8) ? 4 : 8;
    __shared__ __attribute__((aligned(16))) char lds[kWavesPerBlock * kDecWaveLds];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    char* wl = lds + wave * kDecWaveLds;
    const uint32_t cube0 = (blockIdx.x * kWavesPerBlock + wave) * CPW;
    if (cube0 >= n_cubes) return;  // wave-uniform
    {
        int4 v[8];
        dec_load_tile_p<D>((const char*)in, n_cubes, cube0, lane, v);
        dec_stage_tile<D>(wl, lane, v);
    }
    wave_lds_sync();
    const int h = (lane >> 4) & 1, k = lane & (D - 1);
    const int c = (lane >> 5) * (CPW / 2) + ((lane & 15) / D);
    const uint32_t g = cube0 + c;

    // layout A: lane (c, z = k, h) holds face k, rows y, x = 4h + e
    double b[8][4];
    {
        const char* src = wl + c * G::SA_C + k * G::SA_F + h * 16;
        float4 raw[8];
#pragma unroll
        for (int y = 0; y < 8; y++) raw[y] = *(const float4*)(src + y * 32);
#pragma unroll
        for (int y = 0; y < 8; y++) {
            b[y][0] = raw[y].x; b[y][1] = raw[y].y; b[y][2] = raw[y].z; b[y][3] = raw[y].w;
        }
    }
    // pass Y
#pragma unroll
    for (int e = 0; e < 4; e++) {
        double col[8];
#pragma unroll
        for (int y = 0; y < 8; y++) col[y] = b[y][e];
        pin(col);
        f64_line8<INV>(col);
        pin(col);
#pragma unroll
        for (int y = 0; y < 8; y++) b[y][e] = col[y];
    }
    // A -> B: lane-pair swap of the off-diagonal 4x4 blocks
#pragma unroll
    for (int r = 0; r < 4; r++)
#pragma unroll
        for (int e = 0; e < 4; e++) swap16(b[r][e], b[4 + r][e]);
    // pass X
#pragma unroll
    for (int r = 0; r < 4; r++) {
        double row[8];
#pragma unroll
        for (int e = 0; e < 4; e++) {
            row[e] = b[r][e];
            row[4 + e] = b[4 + r][e];
        }
        pin(row);
        f64_line8<INV>(row);
        pin(row);
#pragma unroll
        for (int e = 0; e < 4; e++) {
            b[r][e] = row[e];
            b[4 + r][e] = row[4 + e];
        }
    }
    double cz[D][NXC];
    dec_b_to_c<D>(b, cz, wl, c, k, h);
    // pass Z
#pragma unroll
    for (int e = 0; e < NXC; e++) {
        double col[D];
#pragma unroll
        for (int z = 0; z < D; z++) col[z] = cz[z][e];
        pin(col);
        if constexpr (INV) idctN<D>(col);
        else fdctN<D, false, false>(col, 0.0);
        pin(col);
#pragma unroll
        for (int z = 0; z < D; z++) cz[z][e] = col[z];
    }
    if (g < n_cubes) {
        const int y = (D == 8) ? k : (4 * h + k);
        const int x0 = (D == 8) ? 4 * h : 0;
        float* o = out + (size_t)g * G::CS + y * 8 + x0;
#pragma unroll
        for (int z = 0; z < D; z++) {
            float v[NXC];
#pragma unroll
            for (int e = 0; e < NXC; e++) {
                double t = cz[z][e];
                if constexpr (INV) t = t > 255.0 ? 255.0 : (t < 0.0 ? 0.0 : t);  // 3dDCT.cl:257-261
                v[e] = (float)t;
            }
#pragma unroll
            for (int e = 0; e < NXC; e += 4) *(float4*)(o + z * 64 + e) = make_float4(v[e], v[e + 1], v[e + 2], v[e + 3]);
        }
    }
}

int launch_cube_f32(int D, bool inverse, const float* in, float* out, uint32_t n_cubes, hipStream_t st) {
    const uint32_t per = (D == 8 ? DecGeom<8>::CPW : DecGeom<4>::CPW) * kWavesPerBlock;
    const uint32_t blocks = (n_cubes + per - 1) / per;
    if (!blocks) return 0;
    if (D == 8) {
        if (inverse) hipLaunchKernelGGL((cube_f32_kernel<8, true>), dim3(blocks), dim3(kBlock), 0, st, in, out, n_cubes);
        else hipLaunchKernelGGL((cube_f32_kernel<8, false>), dim3(blocks), dim3(kBlock), 0, st, in, out, n_cubes);
    } else {
        if (inverse) hipLaunchKernelGGL((cube_f32_kernel<4, true>), dim3(blocks), dim3(kBlock), 0, st, in, out, n_cubes);
        else hipLaunchKernelGGL((cube_f32_kernel<4, false>), dim3(blocks), dim3(kBlock), 0, st, in, out, n_cubes);
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Fused stream -> raster decode (dct3d_decode_eg_dev; decoder.c:209-295 after the inflate): the
// wave's CPW cubes are the 2,048 consecutive stream values at marks m0 .. m0 + 63 (the stream decoder's
// mark pass: bit position of every 32nd value).  The wave stages its bit range in its LDS region, lane
// l parses the 32 values from mark m0 + l into registers, the region then receives them at their
// diagonal positions in the decode's staging layout (face-padded cube-major), and decode_tile runs as
// in decode_kernel.  No int32 cube-major array is written or read.
template <int D>
__global__ __launch_bounds__(kBlock, 4) void decode_eg_kernel(DecodeParams P, EgDecParams E) {
    using G = DecGeom<D>;
    constexpr uint32_t CS = G::CS, PARTS = CS / 32, CPW = G::CPW;
    static_assert(CPW * CS == 2048 && PARTS * CPW == 64, "one wave = 64 marks");
    __shared__ __attribute__((aligned(16))) char lds[kWavesPerBlock * kDecWaveLds];
    __shared__ uint16_t s_diag[CS];
    if (E.status[2] != 0) return;  // corrupt / short stream: reported by the mark pass (block-uniform)
    {  // both loads in flight before the LDS writes
        static_assert(CS % kBlock == 0, "whole passes");
        uint16_t t[CS / kBlock];
#pragma unroll
        for (uint32_t r = 0; r < CS / kBlock; r++) t[r] = E.diag[threadIdx.x + r * kBlock];
#pragma unroll
        for (uint32_t r = 0; r < CS / kBlock; r++) s_diag[threadIdx.x + r * kBlock] = t[r];
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    char* wl = lds + wave * kDecWaveLds;
    const uint32_t cube0 = P.cube_base + (blockIdx.x * kWavesPerBlock + wave) * CPW;
    if (cube0 >= P.n_cubes) return;
    const uint64_t n_marks = E.n_values / 32;
    const uint64_t m0 = (uint64_t)cube0 * CS / 32;
    const bool lv = m0 + lane < n_marks;
    const uint64_t my = lv ? E.mark[m0 + lane] : 0;
    const uint64_t first = __shfl(my, 0, 64);
    const uint64_t last = m0 + 64 < n_marks ? E.mark[m0 + 64] : E.status[1];  // wave-uniform
    const uint64_t w0 = first >> 5;
    const uint64_t span = (last >> 5) + 4 - w0;
    constexpr uint32_t WIN = kDecWaveLds / 4;  // 2,304 words >= 2,048 values x 27 bits
    const bool fits = span <= WIN;  // wave-uniform; else the parse reads global memory (parse_values)
    const uint32_t nwin = (uint32_t)(fits ? span : 0);
    uint32_t* win = (uint32_t*)wl;
    // 4 words per lane per round, all loads issued before the first LDS write: a one-word loop waited
    // out a full global round trip per 64 words (3 for ramp content, 6+ for noise)
    // (an empty stream never gets here: the mark pass reported it, status[2]; the guard keeps the
    // clamped index below in range regardless, outside the loop so the loads stay unconditional)
    const uint32_t nst = E.n_words ? nwin : 0u;
    for (uint32_t i0 = 0; i0 < nst; i0 += 256) {
        uint32_t t[4];
#pragma unroll
        for (int b = 0; b < 4; b++) {
            const uint32_t i = i0 + b * 64 + lane;
            t[b] = E.words[min(w0 + i, E.n_words - 1)];  // unconditional (a load under a branch is waited at the join)
        }
#pragma unroll
        for (int b = 0; b < 4; b++) {
            const uint32_t i = i0 + b * 64 + lane;
            if (i < nwin) win[i] = w0 + i < E.n_words ? __builtin_bswap32(t[b]) : 0u;
        }
    }
    wave_lds_sync();
    int32_t v[32];
    parse_values<32>(E, win, nwin, w0, fits, my, v);
    wave_lds_sync();
    {
        const uint32_t c = lane / PARTS, part = lane % PARTS;
        char* cb = wl + c * G::SA_C;
#pragma unroll
        for (int i = 0; i < 32; i++) {
            const uint32_t k = s_diag[part * 32 + i];
            *(int32_t*)(cb + (k >> 6) * G::SA_F + (k & 63) * 4) = v[i];
        }
    }
    wave_lds_sync();
    decode_tile<D, 1>(P, wl, lane, cube0, [] {});
}

// DIAGNOSTIC variants (DCT3D_DEC_VARIANT=7 / 8; the output is NOT a decode): MODE 1 = memory only
// (the same loads, staging and raster stores, no transform), MODE 2 = compute only (no global loads;
// stores suppressed by a runtime condition).  They split the kernel's time into its memory and compute
// parts (1.9 ms / 1.8 ms against 2.25 ms for the full kernel, c3).
template <int D, int MODE>
__global__ __launch_bounds__(kBlock, 4) void decode_kernel_diag(DecodeParams P) {
    __shared__ __attribute__((aligned(16))) char lds[kWavesPerBlock * kDecWaveLds];
    using G = DecGeom<D>;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    char* wl = lds + wave * kDecWaveLds;
    const uint32_t cube0 = (blockIdx.x * kWavesPerBlock + wave) * G::CPW;
    int4 v[8];
    if (MODE == 2) {
        for (int t = 0; t < 8; t++) v[t] = make_int4(lane + t, (int)cube0 & 7, t, 1);
    } else {
        dec_load_tile<D>(P, cube0, lane, v);
    }
    dec_stage_tile<D>(wl, lane, v);
    wave_lds_sync();
    if (MODE == 1) {
        const int h = (lane >> 4) & 1, k = lane & (D - 1);
        const int c = (lane >> 5) * (G::CPW / 2) + ((lane & 15) / D);
        const uint32_t g = cube0 + c;
        uint32_t acc = 0;
        for (int ky = 0; ky < 8; ky++) {
            const int4 x = *(const int4*)(wl + c * G::SA_C + k * G::SA_F + h * 16 + ky * 32);
            acc += x.x ^ x.y ^ x.z ^ x.w;
        }
        if (g < P.n_cubes) {
            const uint32_t s = g / P.cubes_per_stack, rr = g - s * P.cubes_per_stack;
            const uint32_t by = rr / P.nbx, bx = rr - by * P.nbx;
            uint8_t* dst = P.out + (size_t)s * P.stack_stride + (size_t)(by * 8 + k) * P.width + bx * 8 + 4 * h;
            for (int z = 0; z < D; z++) *(uint32_t*)(dst + (size_t)z * P.plane) = acc + z;
        }
        return;
    }
    DecodeParams Q = P;
    if (MODE == 2 && P.width != 0xFFFFFFFFu) Q.n_cubes = 0;  // all stores suppressed, compute kept
    decode_tile<D, 1>(Q, wl, lane, cube0, [] {});
}

// Exact Java InverseDCT fold (InverseDCT.java:56-66: k ascending, zero coefficients skipped, then
// clamp and truncation) for uncertified pixels.
//   per-pixel entries (flag list; the 8-lanes-per-cube decode variant): one thread per entry;
//   whole-cube entries (cube list): one block per cube, its dequantised coefficients in LDS (the
//   zero test is block-uniform), thread t folds pixels t and t + 256 with coalesced table reads.
__device__ __forceinline__ void store_decoded(const DecodeFixupParams& P, uint32_t g, int n, double acc) {
    const double mn = acc < 255.0 ? acc : 255.0;
    const double v = mn > 0.0 ? mn : 0.0;
    const uint32_t s = g / P.cubes_per_stack;
    const uint32_t r = g - s * P.cubes_per_stack;
    const uint32_t by = r / P.nbx, bx = r - by * P.nbx;
    const int z = n / 64, y = (n / 8) & 7, x = n & 7;
    P.out[(size_t)s * P.stack_stride + (size_t)z * P.plane + (size_t)(by * 8 + y) * P.width + bx * 8 + x] =
        (uint8_t)(int)v;
}

template <int D>
__global__ __launch_bounds__(256) void decode_fixup_kernel(DecodeFixupParams P) {
    constexpr int CS = 64 * D;
    __shared__ double cf[CS];
    const uint32_t nf = min(P.counters[0], P.flag_cap);
    const uint32_t ncube = P.counters[1];
    for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < nf; e += gridDim.x * blockDim.x) {
        const unsigned long long v = P.flag_list[e];
        const uint32_t g = (uint32_t)(v / CS);
        const int n = (int)(v % CS);
        const int32_t* q = P.in + (size_t)g * CS;
        double acc = 0.0;
        for (int k = 0; k < CS; k++) {
            const int32_t qk = q[k];
            if (qk != 0) {
                const int kz = k / 64, ky = (k / 8) & 7, kx = k & 7;
                const double c = (double)qk * (double)max(1, 5 * (kx + ky + kz));
                acc = __dadd_rn(acc, __dmul_rn(c, P.inv_coef_t[(size_t)k * CS + n]));  // InverseDCT.java:64
            }
        }
        store_decoded(P, g, n, acc);
    }
    for (uint32_t ci = blockIdx.x; ci < ncube; ci += gridDim.x) {
        const uint32_t g = P.cube_list[ci];
        __syncthreads();
        if (P.in) {
            for (int k = threadIdx.x; k < CS; k += blockDim.x) {
                const int kz = k / 64, ky = (k / 8) & 7, kx = k & 7;
                cf[k] = (double)P.in[(size_t)g * CS + k] * (double)max(1, 5 * (kx + ky + kz));
            }
        } else if (threadIdx.x < CS / 32) {  // fused stream decode: re-parse the cube at its marks
            BitReader<GlobalBits> r{GlobalBits{P.words, P.n_words}, 0, 0, 0, 0};
            r.seek(P.mark[(uint64_t)g * (CS / 32) + threadIdx.x]);
            for (int i = 0; i < 32; i++) {
                uint32_t code = 1u;
                (void)r.get(code);
                const int k = P.diag[threadIdx.x * 32 + i];
                const int kz = k / 64, ky = (k / 8) & 7, kx = k & 7;
                cf[k] = (double)eg_value(code) * (double)max(1, 5 * (kx + ky + kz));
            }
        }
        __syncthreads();
        double acc[CS / 256];
#pragma unroll
        for (int i = 0; i < CS / 256; i++) acc[i] = 0.0;
        for (int k = 0; k < CS; k++) {
            const double c = cf[k];
            if (c != 0.0) {
#pragma unroll
                for (int i = 0; i < CS / 256; i++)
                    acc[i] = __dadd_rn(acc[i], __dmul_rn(c, P.inv_coef_t[(size_t)k * CS + threadIdx.x + 256 * i]));
            }
        }
#pragma unroll
        for (int i = 0; i < CS / 256; i++) store_decoded(P, g, threadIdx.x + 256 * i, acc[i]);
    }
}

// =============================================================================================
// Synthetic frames (integer-only, reproducible on host)
// =============================================================================================
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    uint64_t z = x;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void synth_kernel(uint8_t* out, int width, int height, long long n_pix, uint64_t seed,
                                                     long long frame0, int kind) {
    const long long plane = (long long)width * height;
    for (long long base = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 16; base < n_pix;
         base += (long long)gridDim.x * blockDim.x * 16) {
        uint32_t w[4] = {0, 0, 0, 0};
        for (int i = 0; i < 16 && base + i < n_pix; i++) {
            const long long p = base + i;
            const long long f = p / plane + frame0;
            const long long rem = p % plane;
            const int y = (int)(rem / width), x = (int)(rem % width);
            const uint64_t idx = (uint64_t)(frame0 * plane + p);
            const uint64_t h = splitmix64(seed ^ idx);
            int v;
            if (kind == 1) v = (int)(h & 255u);
            else {
                v = 128 + (int)((3ll * x + 5ll * y + 7ll * f) & 63) - 32 + (int)(h & 15u);
                v = v < 0 ? 0 : (v > 255 ? 255 : v);
            }
            w[i >> 2] |= (uint32_t)v << (8 * (i & 3));
        }
        if (base + 16 <= n_pix) {
            *(uint4*)(out + base) = make_uint4(w[0], w[1], w[2], w[3]);
        } else {
            for (int i = 0; base + i < n_pix; i++) out[base + i] = (uint8_t)(w[i >> 2] >> (8 * (i & 3)));
        }
    }
}

// =============================================================================================
// Bandwidth calibration: the encode's traffic mix without the transform.  mode 0: read n_px bytes,
// write 4*n_px (1:4, NT); mode 1: copy (NT); mode 2: write-only 4*n_px (NT); mode 3: read-only.
// =============================================================================================
__global__ __launch_bounds__(256) void ceiling_kernel(const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                                       long long n_px, int mode, unsigned* sink) {
    // Pure streaming, every wave-instruction a contiguous 1 KiB: per iteration a thread reads 4
    // 16-byte chunks (4 loads in flight) and writes 16 (mix 1:4), 4 (copy) or 16 (write-only).
    const long long T = (long long)gridDim.x * blockDim.x;
    const long long g = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long n_in = n_px / 16;
    unsigned acc = 0;
    for (long long it = 0; it * 4 * T < n_in; it++) {
        uint4 v[4];
        if (mode != 2 && mode != 5) {
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const long long c = it * 4 * T + u * T + g;
                if (c < n_in) {
                    const i32x4_t t = __builtin_nontemporal_load((const i32x4_t*)(in + c * 16));
                    v[u] = make_uint4((unsigned)t.x, (unsigned)t.y, (unsigned)t.z, (unsigned)t.w);
                } else {
                    v[u] = make_uint4(0, 0, 0, 0);
                }
            }
        } else {
#pragma unroll
            for (int u = 0; u < 4; u++) v[u] = make_uint4((unsigned)it, (unsigned)g, u, 0);
        }
        if (mode == 0 || mode == 2) {
#pragma unroll
            for (int w = 0; w < 16; w++) {
                const long long o = it * 16 * T + w * T + g;
                const uint4 x = v[w & 3];
                if (o < 4 * n_in) store16<true>(out + o * 16, make_int4((int)x.x, (int)x.y, (int)x.z, (int)(x.w + w)));
            }
        } else if (mode == 1 || mode == 4) {
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const long long c = it * 4 * T + u * T + g;
                const int4 o = make_int4((int)v[u].x, (int)v[u].y, (int)v[u].z, (int)v[u].w);
                if (c < n_in) {
                    if (mode == 1) store16<true>(out + c * 16, o);
                    else *(int4*)(out + c * 16) = o;
                }
            }
        } else if (mode == 5) {
#pragma unroll
            for (int w = 0; w < 16; w++) {
                const long long o = it * 16 * T + w * T + g;
                if (o < 4 * n_in) *(int4*)(out + o * 16) = make_int4((int)it, (int)g, w, 0);
            }
        } else {
#pragma unroll
            for (int u = 0; u < 4; u++) acc += v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
        }
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

int launch_ceiling(const uint8_t* in, uint8_t* out, long long n_px, int mode, unsigned* sink, hipStream_t st) {
    static int grid = -1;
    if (grid < 0) {
        const char* e = getenv("DCT3D_PROBE_GRID");  // calibration knob: blocks of 256 threads
        grid = e ? atoi(e) : 16384;  // best of the 1024..16384 sweep (profiles/r01/probe_sweep.txt)
    }
    hipLaunchKernelGGL(ceiling_kernel, dim3(grid), dim3(256), 0, st, in, out, n_px, mode, sink);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// =============================================================================================
// Launchers
// =============================================================================================
// Encode: 8x8x8 = encode16_kernel (16 lanes per cube, in-wave exact replay, one launch per call);
// 8x8x4 = encode_kernel<4> (8 lanes per cube, flag list + encode_fixup_kernel).  Both store the int32
// output non-temporally.  The variants that lost (8 lanes per cube at 8x8x8, plain stores, NT loads,
// LDS-padded occupancy) are recorded in profiles/r01/encode_variant_sweep.txt, not built.
namespace {
template <int D>
void launch_enc_eg_t(const EncodeParams& P, const EgFusedParams& E, bool sp, hipStream_t st) {
    const uint32_t groups = (P.n_cubes + kCubesPerWave - 1) / kCubesPerWave;
    const uint32_t blocks = (groups + kWavesPerBlock - 1) / kWavesPerBlock;
    if (sp) hipLaunchKernelGGL((encode_eg_kernel<D, true>), dim3(blocks), dim3(kBlock), 0, st, P, E);
    else hipLaunchKernelGGL((encode_eg_kernel<D, false>), dim3(blocks), dim3(kBlock), 0, st, P, E);
}
template <bool MEM>
void launch_enc16(const EncodeParams& P, hipStream_t st) {
    const uint32_t groups = (P.n_cubes - P.g_base + kE16CPW - 1) / kE16CPW;
    const uint32_t blocks = (groups + kWavesPerBlock - 1) / kWavesPerBlock;
    hipLaunchKernelGGL((encode16_kernel<true, MEM>), dim3(blocks), dim3(kBlock), 0, st, P);
}
}  // namespace

bool encode_replays_inwave(int D) { return D == 8; }

int launch_encode(int D, const EncodeParams& P, hipStream_t st) {
    if (P.n_cubes == 0) return 0;
    if (D == 8) {
        launch_enc16<false>(P, st);
    } else {
        const uint32_t groups = (P.n_cubes - P.g_base + kCubesPerWave - 1) / kCubesPerWave;
        const uint32_t blocks = (groups + kWavesPerBlock - 1) / kWavesPerBlock;
        hipLaunchKernelGGL((encode_kernel<4, true>), dim3(blocks), dim3(kBlock), 0, st, P);
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_encode_memonly(int D, const EncodeParams& P, hipStream_t st) {
    if (P.n_cubes == 0) return 0;
    if (D == 8) {  // the twin of encode16_kernel
        launch_enc16<true>(P, st);
    } else {
        const uint32_t groups = (P.n_cubes + kCubesPerWave - 1) / kCubesPerWave;
        const uint32_t blocks = (groups + kWavesPerBlock - 1) / kWavesPerBlock;
        hipLaunchKernelGGL((encode_memonly_kernel<4>), dim3(blocks), dim3(kBlock), 0, st, P);
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_encode_eg(int D, const EncodeParams& P, const EgFusedParams& E, bool single_pass, hipStream_t st) {
    if (P.n_cubes == 0) return 0;
    if (D == 8) launch_enc_eg_t<8>(P, E, single_pass, st);
    else launch_enc_eg_t<4>(P, E, single_pass, st);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_encode_fixup(int D, const FixupParams& P, int grid, hipStream_t st) {
    if (D != 4) return -1;  // 8x8x8 replays inside encode16_kernel
    hipLaunchKernelGGL(encode_fixup_kernel<4>, dim3(grid), dim3(256), 0, st, P);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

template <int PG>
static void launch_dec_t(int D, uint32_t groups, const DecodeParams& P, hipStream_t st) {
    if (D == 8) hipLaunchKernelGGL((decode_kernel<8, PG>), dim3(groups), dim3(kBlock), 0, st, P);
    else hipLaunchKernelGGL((decode_kernel<4, PG>), dim3(groups), dim3(kBlock), 0, st, P);
}

int launch_decode(int D, const DecodeParams& P, hipStream_t st) {
    if (P.n_cubes == 0) return 0;
    static int variant = -1;
    if (variant < 0) {
        const char* e = getenv("DCT3D_DEC_VARIANT");
        variant = e ? atoi(e) : 1;
    }
    const uint32_t per = (D == 8 ? DecGeom<8>::CPW : DecGeom<4>::CPW) * kWavesPerBlock;
    const uint32_t groups = (uint32_t)((P.n_cubes + per - 1) / per);
    // 1: one butterfly per pin group (default); 4: unpinned (pin groups 1/2/4/none measured within
    // 1 %); 7 / 8: diagnostics, memory-only / compute-only (output NOT valid).  Non-temporal dword
    // output stores were 26 % slower (profiles/r01/decode_variant_sweep.txt).
    switch (variant) {
        case 4: launch_dec_t<0>(D, groups, P, st); break;
        case 7: if (D == 8) hipLaunchKernelGGL((decode_kernel_diag<8, 1>), dim3(groups), dim3(kBlock), 0, st, P); break;
        case 8: if (D == 8) hipLaunchKernelGGL((decode_kernel_diag<8, 2>), dim3(groups), dim3(kBlock), 0, st, P); break;
        default: launch_dec_t<1>(D, groups, P, st); break;
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_decode_eg(int D, const DecodeParams& P, const EgDecParams& E, hipStream_t st) {
    if (P.n_cubes == 0) return 0;
    const uint32_t cpw = (D == 8) ? DecGeom<8>::CPW : DecGeom<4>::CPW;
    const uint32_t waves = (P.n_cubes - P.cube_base + cpw - 1) / cpw;  // cube_base: a multiple of cpw
    const uint32_t blocks = (waves + kWavesPerBlock - 1) / kWavesPerBlock;
    if (D == 8) hipLaunchKernelGGL((decode_eg_kernel<8>), dim3(blocks), dim3(kBlock), 0, st, P, E);
    else hipLaunchKernelGGL((decode_eg_kernel<4>), dim3(blocks), dim3(kBlock), 0, st, P, E);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_decode_fixup(int D, const DecodeFixupParams& P, int grid, hipStream_t st) {
    if (D == 8) hipLaunchKernelGGL(decode_fixup_kernel<8>, dim3(grid), dim3(256), 0, st, P);
    else hipLaunchKernelGGL(decode_fixup_kernel<4>, dim3(grid), dim3(256), 0, st, P);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_synth(uint8_t* out, int width, int height, long long n_pix, uint64_t seed, long long frame0, int kind,
                 hipStream_t st) {
    long long chunks = (n_pix + 15) / 16;
    long long blocks = (chunks + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(synth_kernel, dim3((unsigned)blocks), dim3(256), 0, st, out, width, height, n_pix, seed,
                       frame0, kind);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace dct3d
