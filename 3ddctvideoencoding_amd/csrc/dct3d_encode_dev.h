// dct3d_encode_dev.h -- the encode kernels' device code (templates): rows -> transform -> quantise +
// certify -> staged stores, the exact Java fold and the second certificate.  Instantiated by
// dct3d_kernels.hip (the product) and, for its memory-only twin, dct3d_diag.hip.
#pragma once
#include "dct3d_dev.h"

namespace dct3d {

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
// Descending rows (ky = 7 .. 0; e16_body): the first row reads its NB entries, each later row the one
// entry that enters the window.
template <int NB, int NI>
__device__ __forceinline__ void tab_window_desc(const float4* tab, int& sz, int ky, float A, float (&rr)[NI],
                                                float (&thr)[NI]) {
    asm volatile("" : "+v"(sz));
    const int hi = ky == 7 ? ky + NB - 1 : ky;
#pragma unroll
    for (int i = ky; i <= hi; i++) {
        const float* t = (const float*)(tab + sz + i);
        rr[i] = t[0];
        thr[i] = __builtin_fmaf(-A, t[1], t[2]);
    }
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

// 8x8x4 exact Java fold of the coefficients the certificate left open (exact ties: the 4-point k = 2
// basis row is +-1/2, so (kz = 2, ky, kx in {0, 4}) values can be rational x.5 exactly -- about one
// coefficient in 10^4 on ramp content), the wave's 8 cubes in parallel.  Per round, the 8 lanes of
// cube c take one of its open coefficients k (DCT.java:44-52): lane j sums its row (y = j of frames
// 0..3, px) into the cube's group sums by LDS integer atomics (exact), forms the products of groups
// j, j + 8, ... (one correctly rounded fp64 multiply each, as in Java), and lane 0 of the cube folds
// them in HashMap order, divides by the step and rounds (Math.round), writing the result over the
// stored value.  Rounds = the most open coefficients of any one cube (the whole-wave exact_coef of
// encode16_kernel runs one coefficient per round).  Scratch: the wave's staging region, free again
// after the stores: kGM4 int sums + kGM4 fp64 products per cube.
constexpr int kGM4 = kGM4Dev;  // >= the most Java groups of any 8x8x4 coefficient (40; the plan checks it)
static_assert(8 * kGM4 * (4 + 8) <= enc_wave_lds<4>(), "8x8x4 replay scratch fits the wave's region");
__device__ __forceinline__ void enc4_replay(const EncodeParams& P, const uint2 (&px)[4], uint32_t fm, char* wl,
                                            int lane, uint32_t cube0) {
    constexpr int CS = 256;
    const int c = lane >> 3, j = lane & 7;
    int* const ssum = (int*)wl + c * kGM4;
    double* const prod = (double*)(wl + 8 * kGM4 * 4) + c * kGM4;
    uint32_t nrep = 0;
    for (;;) {
        const uint64_t who = __ballot(fm != 0u);
        if (who == 0ull) break;
        const uint32_t mine = (uint32_t)(who >> (8 * c)) & 0xFFu;  // lanes of this cube still open
        const bool act = mine != 0u;
        const int src = 8 * c + (act ? __builtin_ctz(mine) : 0);
        const int bit = __shfl(fm ? __builtin_ctz(fm) : 0, src, 64);
        const int sj = src & 7;
        const int kz = sj >> 1, ky = bit >> 2, kx = (sj & 1) * 4 + (bit & 3);
        const uint32_t k = (uint32_t)((kz * 8 + ky) * 8 + kx);
        // (lean: loops rolled and the coefficients loaded where used -- an unrolled body cost 20 VGPRs
        // over the whole kernel, i.e. occupancy)
        int ng = 0;
        uint2 gr[4];
        if (act) {
            ng = P.ngroups[k];
#pragma unroll
            for (int z = 0; z < 4; z++) gr[z] = *(const uint2*)(P.group_of + (size_t)k * CS + (z * 8 + j) * 8);
#pragma unroll 1
            for (int i = j; i < kGM4; i += 8) ssum[i] = 0;
        }
        wave_lds_sync();
        if (act) {
#pragma unroll
            for (int z = 0; z < 4; z++) {
                const uint2 gz = gr[z], pz = px[z];
#pragma unroll
                for (int e = 0; e < 4; e++) {
                    const int g0 = (int)((gz.x >> (8 * e)) & 0xFFu), g1 = (int)((gz.y >> (8 * e)) & 0xFFu);
                    if (g0 < ng) atomicAdd(&ssum[g0], (int)((pz.x >> (8 * e)) & 0xFFu));
                    if (g1 < ng) atomicAdd(&ssum[g1], (int)((pz.y >> (8 * e)) & 0xFFu));
                }
            }
        }
        wave_lds_sync();
        if (act) {
#pragma unroll 1
            for (int i = j; i < ng; i += 8)
                prod[i] = __dmul_rn((double)ssum[i], P.coef[(size_t)k * kMaxGroupsDev + i]);
        }
        wave_lds_sync();
        if (act && j == 0) {
            double acc = 0.0;
#pragma unroll 1
            for (int gi = 0; gi < ng; gi++) acc = __dadd_rn(acc, prod[gi]);  // DCT.java:50, in order
            const int q = java_round_dev(__ddiv_rn(acc, (double)max(1, 5 * (kx + ky + kz))));
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // after the wave's staged stores (one in-order count)
            P.out[(size_t)(cube0 + c) * CS + k] = q;
        }
        nrep += (uint32_t)__builtin_popcountll(__ballot(act && j == 0));
        if (act && lane == src) fm &= fm - 1u;
        wave_lds_sync();  // the next round rewrites the sums
    }
    if (lane == 0 && P.replay_count) atomicAdd(P.replay_count + (blockIdx.x & (kCountSpread - 1)), nrep);
}

// Everything after the row loads, for the 8 cubes from cube0 (8x8x4): statistics, transform, quantise +
// certify, staged 1 KiB stores, the exact fold of the uncertified coefficients (enc4_replay).
template <int D, bool NT>
__device__ __forceinline__ void encode_body(const EncodeParams& P, const uint2 (&raw)[D], char* wl,
                                            const float4* tab, int lane, uint32_t cube0) {
    static_assert(D == 4, "8x8x8 encodes in encode16_kernel");
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
    // Uncertified coefficients: the lane's mask fm, bit ky * 4 + x (coefficient (kz, ky, kx0 + x)).
    int sz = so;
    float rr[NI], thr[NI];
    int32_t qv[8][NB];
    uint32_t fm = 0u;
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
        if (__builtin_expect(f, 0)) {
            uint32_t bits = 0;
#pragma unroll
            for (int x = 0; x < NB; x++)
                if (__builtin_fabsf(qq[x] - __builtin_rintf(qq[x])) >= thr[ky + x]) bits |= 1u << x;
            fm |= bits << (ky * NB);
        }
        pin(qv[ky]);
        asm volatile("" : "+v"(fm));  // the row's checks complete here (q, n die)
    }
    if (j == 0) {
        qv[0][0] = java_round_dev((double)S * P.coef_dc);  // exact DC (single Java group)
        fm &= ~1u;
    }
    if (!valid) fm = 0u;

    enc_stage_store<D, NT>(P, qv, wl, lane, cube0);

    // rare path: the rows again (after the stores: held across them they cost occupancy), the fold
    if (__builtin_expect(__ballot(fm != 0u) != 0ull, 0)) {  // wave-uniform
        uint2 px[D];
        load_rows<D>(P, g, valid, j, px);
        enc4_replay(P, px, fm, wl, lane, cube0);
    }
}

// One wave = one group of 8 consecutive cubes (register-prefetch loops over several groups spill
// and were 25-40 % slower: profiles/r01/encode_variant_sweep.txt).
template <int D, bool NT, bool NTL = false>
__global__ __launch_bounds__(kBlock, 4) void encode_kernel(EncodeParams P) {
    __shared__ __attribute__((aligned(16))) char lds[kWavesPerBlock * enc_wave_lds<D>()];
    __shared__ float4 s_tab[kTabN];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t cube0 = P.g_base + (xcd_tile<64>() * kWavesPerBlock + wave) * kCubesPerWave;
    uint2 raw[D];
    __builtin_amdgcn_s_setprio(3);
    load_rows<D, NTL>(P, cube0 + (lane >> 3), cube0 + (lane >> 3) < P.n_cubes, lane & 7, raw);  // in flight first
    __builtin_amdgcn_s_setprio(0);
    if (blockIdx.x == 0 && P.replay_clear) {
#pragma unroll
        for (int i = 0; i < 2 * kCountSpread / kBlock; i++) P.replay_clear[i * kBlock + threadIdx.x] = 0u;
    }
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
constexpr int kE16Lds = 4 * kE16TC;
// int16 staging of all 4 cubes at once (|q| <= 255 sqrt(512) < 2^15 by Parseval, DC included): face of
// 8 rows x 8 values (128 B) + 16 B bank spread, so the second certificate settles its coefficients in LDS
// before any store is issued.  (int32 staging, two cubes per round, with the recheck after the stores:
// c2 uniform 2.043 -> 2.018 ms, c2 1.883 -> 1.870 ms; profiles/r03/variant_sweep.txt)
constexpr int kE16S16F = 144;
constexpr int kE16S16C = 8 * kE16S16F;
static_assert(4 * kE16S16C <= kE16Lds, "int16 staging of the wave's 4 cubes fits its region");

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
    // rows and columns in descending order, fm = 2 fm + open: one v_addc per coefficient (the compare's
    // lane mask is the carry-in), and coefficient (ky, e) ends at bit 4 ky + e
#pragma unroll
    for (int ky = 7; ky >= 0; ky--) {
        pin(b[ky]);
        tab_window_desc<4, 11>(tab, sz, ky, A, rr, thr);
#pragma unroll
        for (int e = 3; e >= 0; e--) {
            const float qq = b[ky][e] * rr[ky + e];
            const float n = __builtin_rintf(qq);
            const unsigned long long open = __ballot(__builtin_fabsf(qq - n) >= thr[ky + e]);
            unsigned long long cout;
            asm("v_addc_co_u32_e64 %0, %1, %2, %2, %3" : "=v"(fm), "=s"(cout) : "v"(fm), "s"(open));
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
// Timing: it runs after the wave's cubes are staged as int16 in LDS and before any store is issued, so
// its row reload (L2) waits for nothing but itself; the owning lane writes a settled value over the
// provisional one in the staging (wl).  Register pressure stays with the main path's 72 VGPRs (the
// staged values are out of the registers by then).  s_b: the block's copy of the tables ([64] basis,
// [32] thresholds), written by every wave that takes this path (identical bits) and read only after its
// own writes.
__device__ __forceinline__ void e16_recheck64(const uint2 (&raw)[4], double bv, double tv, double* s_b, char* wl,
                                              int lane, uint32_t& fm, uint32_t& nset) {
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
            // rows picked by selects, not raw[e]: a runtime index would put raw in scratch memory
            const uint2 ra = e == 0 ? raw[0] : raw[2], rb = e == 0 ? raw[1] : raw[3];
            uint32_t w[4] = {ra.x, rb.x, ra.y, rb.y};
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
                const uint32_t cl = (lane >> 5) * 2 + ((lane & 15) >> 3);  // the cube within the wave
                *(int16_t*)(wl + cl * kE16S16C + kz * kE16S16F + (ky * 8 + kx) * 2) = (int16_t)n;  // int16 staging
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

// MODE 1 (dct3d_encode_diag_dev memory only, DIAGNOSTIC: the output is NOT a DCT): the same loads,
// staging and stores with the transform, quantisation and certification replaced by a few integer ops.
// MODE 2 (compute only, DIAGNOSTIC): ramp-like rows made from the lane and cube indices instead of the
// loads, the whole transform / quantise / certify / staging, the stores suppressed by a runtime
// condition (P.width == 0 never holds) and the rare paths skipped, so its time is the kernel's main-path
// issue work alone.
// One launch is the whole encode: no flag list, no counter reset, no fixup launch.  Block 0 zeroes the
// next call's counter slot (P.replay_clear; the two slots alternate between calls).  7 waves per SIMD
// (72 VGPRs) is what the main path needs; the attribute keeps the rare paths from raising it (the
// kernel needs no scratch: tools/isa_count.py).
static_assert(kMaxGroupsDev * (4 + 8) <= kE16Lds, "exact-replay scratch fits the wave's region");
// Diagnostic traversal (MODES 4 / 5): wave slot s, counted strip-major (stack, strip, block row, column in
// the strip), -> the cube it encodes (the reference's cube-major index, so the output is unchanged)
__device__ __forceinline__ uint32_t strip_cube(const EncodeParams& P, uint32_t s) {
    const uint32_t st = fdiv(s, P.div_cps);
    const uint32_t r = s - st * P.cubes_per_stack;
    const uint32_t strip = fdiv(r, P.div_strip_cubes);
    const uint32_t rr = r - strip * P.strip_cubes;
    const uint32_t by = fdiv(rr, P.div_strip_w);
    return st * P.cubes_per_stack + by * P.nbx + strip * P.strip_w + (rr - by * P.strip_w);
}
template <bool NT, int MODE = 0>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(7))) void encode16_kernel(EncodeParams P) {
    constexpr int CS = 512;
    // MODE 4 / 5: MODE 1 / 0 with the strip traversal (diagnostic sweep)
    constexpr bool MEM = MODE == 1 || MODE == 4, COMP = MODE == 2, TRACE = MODE == 3, STRIP = MODE >= 4;
    uint64_t t_start = 0, t_comp = 0;
    if constexpr (TRACE) t_start = __builtin_amdgcn_s_memrealtime();
    __shared__ __attribute__((aligned(16))) char lds[kWavesPerBlock * kE16Lds];
    __shared__ float4 s_tab[kTabN];
    __shared__ double s_b64[96];  // second certificate tables (rare path)
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#ifndef DCT3D_E16_XCD_G  // A/B only: the XCD tile run length of encode16_kernel
#define DCT3D_E16_XCD_G 64
#endif
    const uint32_t slot0 = P.g_base + (xcd_tile<DCT3D_E16_XCD_G>() * kWavesPerBlock + wave) * kE16CPW;
    uint32_t cube0 = slot0;
    if constexpr (STRIP) cube0 = slot0 < P.n_cubes ? strip_cube(P, slot0) : slot0;
    const int k = lane & 7, h = (lane >> 4) & 1;
    const int c = (lane >> 5) * 2 + ((lane & 15) >> 3);
    const uint32_t g = cube0 + c;
    const bool valid = g < P.n_cubes;
    uint2 raw[4];
    if constexpr (COMP) {
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const uint32_t b0 = 96u + 5u * (uint32_t)k + 7u * (uint32_t)(4 * h + r) + (g & 15u);
            raw[r] = make_uint2((b0 * 0x01010101u) + 0x09060300u, (b0 * 0x01010101u) + 0x15120F0Cu);
        }
    } else {
        // a starting wave computes its addresses and issues its loads at the top priority: under the
        // default oldest-first issue they queue behind the computing waves' VALU work, and a box whose
        // encode loses the overlap of memory and compute that way runs 10 % slower (variant_sweep.txt)
        if constexpr (!MEM) __builtin_amdgcn_s_setprio(3);
        e16_load(P, g, valid, k, h, raw);
        if constexpr (!MEM) __builtin_amdgcn_s_setprio(0);
    }
    if (!MEM && !COMP && blockIdx.x == 0 && P.replay_clear) {
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
    if constexpr (TRACE) t_comp = __builtin_amdgcn_s_memrealtime();
    const bool rare = !MEM && !COMP && P.recheck && __builtin_expect(__ballot(fm != 0u) != 0ull, 0);  // wave-uniform

    const ReplayGeom R{P.raster, P.cubes_per_stack, P.nbx, P.width, P.plane, P.stack_stride,
                       P.ngroups, P.coef, P.group_of};

    {
        // ---- all 4 cubes staged as int16 at once; the second certificate settles its coefficients in
        //      this staging (its row reload waits for nothing but itself: no store has been issued yet);
        //      then 8 stores of 1 KiB, each lane's 4 int16 widened to 16 B ----
        {
            char* dst = wl + c * kE16S16C + k * kE16S16F + h * 8;
#pragma unroll
            for (int ky = 0; ky < 8; ky++)
                *(uint2*)(dst + ky * 16) = make_uint2(__builtin_amdgcn_perm(qv[ky][1], qv[ky][0], 0x05040100u),
                                                      __builtin_amdgcn_perm(qv[ky][3], qv[ky][2], 0x05040100u));
        }
        wave_lds_sync();
        if (rare) {
            uint2 raw2[4];
            e16_load(P, g, valid, k, h, raw2);
            const double bv = P.tab64[lane];
            const double tv = lane < 32 ? P.tab64[64 + lane] : 0.0;
            uint32_t nset;
            e16_recheck64(raw2, bv, tv, s_b64, wl, lane, fm, nset);
            for (int o = 1; o < 64; o <<= 1) nset += __shfl_xor(nset, o, 64);
            if (lane == 0 && nset && P.replay_count)
                atomicAdd(P.replay_count + kCountSpread + (blockIdx.x & (kCountSpread - 1)), nset);
        }
        char* outb = (char*)(P.out + (size_t)cube0 * CS);
#pragma unroll
        for (int t = 0; t < 8; t++) {
            const int q = t * 64 + lane;  // 16-byte output chunk of the wave's 4 cubes (4 values)
            const int cc = q >> 7, face = (q >> 4) & 7, w = q & 15;
            if (cube0 + cc < P.n_cubes && (!COMP || P.width == 0u)) {
                const uint2 v = *(const uint2*)(wl + cc * kE16S16C + face * kE16S16F + w * 8);
                store16<NT>(outb + (size_t)q * 16, make_int4((int)(int16_t)v.x, (int)v.x >> 16, (int)(int16_t)v.y,
                                                             (int)v.y >> 16));
            }
        }
        wave_lds_sync();
    }
    if constexpr (TRACE) {  // the wave's timeline: start, transform done, stores issued (+ 100 MHz clock)
        const uint64_t t_end = __builtin_amdgcn_s_memrealtime();
        const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);   // HW_ID
        const uint32_t xcc = __builtin_amdgcn_s_getreg((15 << 11) | (0 << 6) | 20); // XCC_ID
        if (lane == 0) {
            uint64_t* tr = P.trace + (size_t)((cube0 - P.g_base) / kE16CPW) * 4;
            *(ulonglong2*)tr = make_ulonglong2(t_start, t_comp);
            *(ulonglong2*)(tr + 2) = make_ulonglong2(t_end, ((uint64_t)xcc << 32) | hw);
        }
    }

    // ---- rarest path: the exact Java fold of every coefficient both certificates left open (exact
    //      ties, e.g. k = (0, 2, 2) where the basis products lie in Q(sqrt 2) and the value can be a
    //      rational x.5 exactly: a few per 10^8 coefficients), whole wave, one at a time, written over
    //      the stored value by lane 0.  Its loads wait for the wave's stores (one in-order vmcnt), and
    //      lane 0's store follows its own earlier store of that word (vmcnt(0)), so the exact value is
    //      the one that stays. ----
    if (__builtin_expect(!MEM && !COMP && __ballot(fm != 0u) != 0ull, 0)) {
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

}  // namespace dct3d
