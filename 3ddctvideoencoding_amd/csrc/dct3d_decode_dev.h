// dct3d_decode_dev.h -- the decode kernel's device code (templates): staged loads -> dequantise ->
// inverse passes -> certify -> raster stores.  Instantiated by dct3d_kernels.hip (the product) and
// dct3d_diag.hip (the memory-only / compute-only split).
#pragma once
#include "dct3d_dev.h"

namespace dct3d {

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
constexpr int kDecWaveLds = 9280;  // 4 x (8 x 288 + 16) (8x8x8); 4 blocks per CU with the stream decode's s_diag

template <int D>
struct DecGeom {
    static constexpr int CS = 64 * D;
    static constexpr int LPC = 2 * D;          // lanes per cube
    static constexpr int CPW = 64 / LPC;       // cubes per wave: 4 (D=8) | 8 (D=4)
    static constexpr int SA_F = 288;           // staging face stride (256 B + 32 B pad)
    // staging cube stride; 8x8x8: + 16 B so that the wave's cubes start 4 banks apart (the layout-A reads of
    // lanes (c1 = 0, 1) and the stream decode's value scatter over 4 cubes were 2- and 4-way bank conflicts)
    static constexpr int SA_C = D * SA_F + (D == 8 ? 16 : 0);
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

// ---- exact replay of one lane's 32 pixels (InverseDCT.java:56-66 / Decoder.java:107-117: for each pixel,
//      k ascending, zero coefficients skipped, acc = acc + c_k * coef[n][k] with both operations rounded,
//      then clamp to [0, 255] and the (int) / (byte) truncation).  The whole wave: reload() puts the
//      cube's dequantised coefficients in LDS (cf[k] = q_k * step_k, exact), the non-zero k go to an
//      ascending list, then lane p < 32 folds pixel p of lane `src` (layout C: D=8 z = p/4, x = 4h + p%4;
//      D=4 z = p/8, x = p%8), its table reads batched 8 at a time ahead of the sequential fold; the bytes
//      land in LDS in lane src's word order.  A cube's certificate fails at one pixel in practice, so
//      the replay is one lane's 32 pixels, not the cube's 512 (a dense cube's whole-cube fold took
//      ~0.4 ms: a kernel tail).  Not inlined: the main path's register allocation stays its own. ----
template <int D>
struct ReloadCubes {  // from the int32 cube-major input
    const int32_t* in;
    __device__ __forceinline__ void operator()(uint32_t g, double* cf, int lane) const {
        constexpr int CS = 64 * D;
#pragma unroll
        for (int i = 0; i < CS / 64; i++) {
            const int k = lane + 64 * i;
            const int kz = k / 64, ky = (k / 8) & 7, kx = k & 7;
            cf[k] = (double)in[(size_t)g * CS + k] * (double)max(1, 5 * (kx + ky + kz));
        }
    }
};

template <int D, class Reload>
__device__ __attribute__((noinline)) const uint8_t* decode_replay_lane(const double* inv_coef_t, Reload reload,
                                                                       char* wl, int lane, uint32_t g, int src) {
    constexpr int CS = 64 * D, NP = CS / 64, B = 8;
    static_assert(CS * 8 + CS * 2 + 32 <= kDecWaveLds, "replay scratch fits the wave's region");
    double* cf = (double*)wl;
    uint16_t* nzk = (uint16_t*)(wl + CS * 8);
    uint8_t* ob = (uint8_t*)(wl + CS * 10);
    wave_lds_sync();
    reload(g, cf, lane);
    wave_lds_sync();
    // the non-zero coefficients in ascending k (the fold skips zeros: InverseDCT.java:60)
    uint32_t nnz = 0;
#pragma unroll
    for (int i = 0; i < NP; i++) {
        const bool nz = cf[64 * i + lane] != 0.0;
        const unsigned long long bm = __ballot(nz);
        if (nz) nzk[nnz + __builtin_amdgcn_mbcnt_hi((uint32_t)(bm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bm, 0u))] = (uint16_t)(64 * i + lane);
        nnz += (uint32_t)__builtin_popcountll(bm);
    }
    wave_lds_sync();
    if (lane < 32) {
        const int sk = src & (D - 1), sh = (src >> 4) & 1;
        const int y = (D == 8) ? sk : 4 * sh + sk;
        const int z = (D == 8) ? lane >> 2 : lane >> 3;
        const int x = (D == 8) ? 4 * sh + (lane & 3) : lane & 7;
        const double* col = inv_coef_t + (z * 64 + y * 8 + x);  // coef[n][k] at col[k * CS]
        double acc = 0.0;
        for (uint32_t j = 0; j < nnz; j += B) {
            double t[B];
            uint32_t kk[B];
#pragma unroll
            for (int u = 0; u < B; u++) {  // a padded slot (past nnz) re-reads the last k and adds +-0
                kk[u] = nzk[min(j + u, nnz - 1)];
                t[u] = col[(size_t)kk[u] * CS];
            }
#pragma unroll
            for (int u = 0; u < B; u++) {
                const double cv = j + u < nnz ? cf[kk[u]] : 0.0;
                acc = __dadd_rn(acc, __dmul_rn(cv, t[u]));
            }
        }
        const double mn = acc < 255.0 ? acc : 255.0;
        ob[lane] = (uint8_t)(int)(mn > 0.0 ? mn : 0.0);
    }
    wave_lds_sync();
    return ob;
}

// the cube of a lane within its wave (decode layouts: lane = c2*32 + h*16 + c1*D + k)
template <int D>
__device__ __forceinline__ int dec_cube_of_lane(int lane) { return (lane >> 5) * (DecGeom<D>::CPW / 2) + ((lane & 15) / D); }

// ---- stores of one tile's bytes (decode_tile; the memory-only twin in dct3d_diag.hip) ----
// outw[z][wd]: lane (c, y, h)'s bytes of plane z (layout C: D=8 x 4h..4h+3 of row k; D=4 x 0..7 of
// row 4h + k).  A full block (its 4 waves' 4 CPW consecutive cubes all exist; nbx even, so a 16-byte
// pair of cubes never straddles a block-row) leaves through LDS: each wave puts its rows in its own
// region ([z][y][CPW x 8 B]; every earlier use of the region is over), one barrier, then every 16-byte
// chunk of the block's rows -- two cubes of one row of one plane -- goes out with a non-temporal store,
// a wave instruction covering 1 KiB of whole 128-byte lines.  Per-lane 4- or 8-byte row pieces cost
// ~1.5x the write time (profiles/r02/variant_sweep.txt).  Other blocks store per lane.  Every wave of
// the block must call this (the barrier); a full block has no early-returning wave.
// LOOP: called inside a caller's loop (decode_eg_kernel's groups): the lane's addresses are made here, not
// hoisted out of the loop and held across the transform.
template <int D, bool LOOP = false>
__device__ __forceinline__ void dec_store_tile(const DecodeParams& P, char* wl, int lane, uint32_t cube0,
                                               const uint32_t (&outw)[D][(D == 8) ? 1 : 2], bool valid) {
    using G = DecGeom<D>;
    constexpr int CPW = G::CPW;
    constexpr int NXC = (D == 8) ? 4 : 8;
    constexpr int W = CPW * 8;  // bytes of one row of the wave's cubes
    const int h = (lane >> 4) & 1, k = lane & (D - 1);
    const int y = (D == 8) ? k : (4 * h + k);
    const int x0 = (D == 8) ? 4 * h : 0;
    const int c = dec_cube_of_lane<D>(lane);
    const int wave = (int)(threadIdx.x >> 6);
    const uint32_t blk0 = cube0 - (uint32_t)wave * CPW;
    if (P.blk_store && blk0 + kWavesPerBlock * CPW <= P.n_cubes) {  // block-uniform
#pragma unroll
        for (int z = 0; z < D; z++) {
            char* t = wl + z * 8 * W + y * W + c * 8 + x0;
            if constexpr (NXC == 4) *(uint32_t*)t = outw[z][0];
            else *(uint2*)t = make_uint2(outw[z][0], outw[z][1]);
        }
        __syncthreads();
        const char* lds0 = wl - wave * kDecWaveLds;
        constexpr int CPR = kWavesPerBlock * W / 16;  // 16-byte chunks per block row
        int tid = (int)threadIdx.x;
        if constexpr (LOOP) asm volatile("" : "+v"(tid));
        // the block's first cube, wave-uniform (scalar arithmetic); a block inside one block-row (every
        // block when nbx is a multiple of 4 CPW) addresses its chunks from it directly
        const uint32_t b0 = __builtin_amdgcn_readfirstlane(blk0);
        const uint32_t s0 = fdiv(b0, P.div_cps);
        const uint32_t rr0 = b0 - s0 * P.cubes_per_stack;
        const uint32_t by0 = fdiv(rr0, P.div_nbx), bx0 = rr0 - by0 * P.nbx;
        const bool one_row = bx0 + kWavesPerBlock * CPW <= P.nbx;
        uint8_t* const base0 = P.out + (size_t)s0 * P.stack_stride + (size_t)(by0 * 8) * P.width + bx0 * 8;
#pragma unroll
        for (int i = 0; i < D * 8 * CPR / kBlock; i++) {
            const int q = tid + kBlock * i;
            const int z = q / (8 * CPR), r = q % (8 * CPR), yy = r / CPR, j = r % CPR;
            const int4 v = *(const int4*)(lds0 + (j * 16 / W) * kDecWaveLds + z * 8 * W + yy * W + (j * 16) % W);
            uint8_t* dst;
            if (one_row) {
                dst = base0 + ((uint32_t)z * (uint32_t)P.plane + (uint32_t)yy * P.width + (uint32_t)j * 16u);  // < 2^32 within a stack
            } else {
                const uint32_t gc = blk0 + 2 * j;
                const uint32_t s = fdiv(gc, P.div_cps);
                const uint32_t rr = gc - s * P.cubes_per_stack;
                const uint32_t by = fdiv(rr, P.div_nbx), bx = rr - by * P.nbx;
                dst = P.out + (size_t)s * P.stack_stride + (size_t)z * P.plane + (size_t)(by * 8 + yy) * P.width + bx * 8;
            }
            __builtin_nontemporal_store(i32x4_t{v.x, v.y, v.z, v.w}, (i32x4_t*)dst);
        }
    } else if (valid) {
        const uint32_t g = cube0 + c;
        const uint32_t s = fdiv(g, P.div_cps);
        const uint32_t rr = g - s * P.cubes_per_stack;
        const uint32_t by = fdiv(rr, P.div_nbx), bx = rr - by * P.nbx;
        uint8_t* dst = P.out + (size_t)s * P.stack_stride + (size_t)(by * 8 + y) * P.width + bx * 8 + x0;
#pragma unroll
        for (int z = 0; z < D; z++, dst += P.plane) {  // one 64-bit add per plane
            if constexpr (NXC == 4) *(uint32_t*)dst = outw[z][0];
            else *(uint2*)dst = make_uint2(outw[z][0], outw[z][1]);
        }
    }
}

// One tile (CPW cubes) from the staged input in the wave's LDS region to the raster.  after_a() runs
// once the staged input is in registers (the persistent variant issues the next tile's loads there);
// reload(g, cf, lane) re-reads cube g's dequantised coefficients for the rare exact replay.
// PG: butterflies per pin group (1: one at a time, 2 / 4: that many interleaved, 0: no pins)
// CODES: the staging holds Exp-Golomb codes, not values (decode_eg_kernel): v = code >> 1, negative when the
// code is odd.  |q| * step in 32-bit integers (v_mul_u32_u24: exact while |q| < 2^15, < 2^22), the lane's
// L1 as their exact integer sum (< 2^27), the fp64 value by one exact conversion with the sign put into its
// sign bit (one v_lshl_or): the same cf as the fp64 product, except that code 1 (value 0) gives -0.0 (the
// outputs' truncation and certificate do not see a zero's sign), at 4 fewer VALU cycles per value than an
// fp64 product and fp64 L1 sum.  A lane holding a code >= 2^16 (|q| >= 2^15: a code of 33+ bits, never
// written for 8-bit frames) reports L1 = inf, so its whole cube goes to the exact replay, which reloads the
// values from the stream.
template <int D, int PG, bool LOOP = false, bool CODES = false, class AfterA, class Reload>
__device__ __forceinline__ void decode_tile(const DecodeParams& P, char* wl, int lane, uint32_t cube0,
                                            AfterA&& after_a, const Reload& reload) {
    using G = DecGeom<D>;
    constexpr int CPW = G::CPW;
    constexpr int NXC = (D == 8) ? 4 : 8;  // x values per lane in layout C
    const int h = (lane >> 4) & 1;
    const int k = lane & (D - 1);
    const int c = (lane >> 5) * (CPW / 2) + ((lane & 15) / D);
    const uint32_t g = cube0 + c;
    const bool valid = g < P.n_cubes;

    // ---- layout A: dequantise, L1 ----
    // cf = q * step in fp64: an exact conversion and an exact product (|q * step| < 2^38) for every int32
    // q.  L1 = sum |cf| over the cube bounds both the error (|v - v_java| <= dec_G L1 + dec_E) and the
    // values (|v| <= Bmax L1): one fp64 add per value (|x| is a source modifier), summed over the lane,
    // then over the cube's lanes in fp32 with a final factor that covers every rounding on the way
    // (fp64 sum 2^-48, the conversion and five fp32 roundings 6 * 2^-24 < 2^-19).
    double b[8][4];
    float l1_f;
    {
        int sb = 5 * (4 * h + k);  // step = sb + 5 (e + ky); DC (e = ky = 0): 1
        if constexpr (LOOP) asm volatile("" : "+v"(sb));  // (dec_store_tile's LOOP)
        const char* src = wl + c * G::SA_C + k * G::SA_F + h * 16;
        int4 raw[8];  // all eight LDS reads in flight before the first use
#pragma unroll
        for (int ky = 0; ky < 8; ky++) raw[ky] = *(const int4*)(src + ky * 32);
        if constexpr (CODES) {
            uint32_t l1 = 0, any = 0;
#pragma unroll
            for (int ky = 0; ky < 8; ky++) {
                const uint32_t vv[4] = {(uint32_t)raw[ky].x, (uint32_t)raw[ky].y, (uint32_t)raw[ky].z, (uint32_t)raw[ky].w};
                any |= vv[0] | vv[1] | vv[2] | vv[3];
#pragma unroll
                for (int e = 0; e < 4; e++) {
                    const uint32_t st = (e + ky) ? (uint32_t)(sb + 5 * (e + ky)) : (uint32_t)max(sb, 1);
                    const uint32_t ms = __umul24(vv[e] >> 1, st);  // |q| * step
                    l1 += ms;
                    uint2 m = __builtin_bit_cast(uint2, (double)ms);
                    asm("v_lshl_or_b32 %0, %1, 31, %2" : "=v"(m.y) : "v"(vv[e]), "v"(m.y));  // the sign: the code odd
                    b[ky][e] = __builtin_bit_cast(double, m);
                }
            }
            l1_f = any < 0x10000u ? (float)l1 : __builtin_inff();
        } else {
            double stp[11];
            stp[0] = (double)max(sb, 1);
#pragma unroll
            for (int j = 1; j < 11; j++) stp[j] = (double)(sb + 5 * j);
            double l1 = 0.0;
#pragma unroll
            for (int ky = 0; ky < 8; ky++) {
                const int vv[4] = {raw[ky].x, raw[ky].y, raw[ky].z, raw[ky].w};
#pragma unroll
                for (int e = 0; e < 4; e++) {
                    b[ky][e] = __dmul_rn((double)vv[e], stp[e + ky]);
                    l1 = __dadd_rn(l1, __builtin_fabs(b[ky][e]));
                }
            }
            l1_f = (float)l1;
        }
    }
    after_a();
    // L1 over the cube's lanes (k bits, then bit 4): DPP within the row, one permlane16 swap across
    l1_f += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, l1_f), 0xB1, 0xF, 0xF, false));  // quad_perm xor 1
    l1_f += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, l1_f), 0x4E, 0xF, 0xF, false));  // quad_perm xor 2
    if constexpr (D == 8)
        l1_f += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, l1_f), 0x141, 0xF, 0xF, false));  // row_half_mirror
    {
        const auto sw = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(uint32_t, l1_f), __builtin_bit_cast(uint32_t, l1_f), false, false);
        l1_f = (__builtin_bit_cast(float, (uint32_t)sw[0]) + __builtin_bit_cast(float, (uint32_t)sw[1])) * (1.0f + 0x1p-19f);
    }

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
        for (int i = 0; i < G3; i++) idctN_fix<D>(col[i], kFixMagic);  // outputs v + kFixMagic
        if (PG) for (int i = 0; i < G3; i++) pin(col[i]);
#pragma unroll
        for (int i = 0; i < G3; i++)
#pragma unroll
            for (int z = 0; z < D; z++) cz[z][e0 + i] = col[i][z];
    }

    // ---- certify, clamp + truncate, store ----
    // |v - v_java| <= m = dec_G L1 + dec_E (dct3d_plan.cpp).  The byte is clamp(floor(v), 0, 255),
    // monotone in v, so it is Java's byte when floor is constant over [v - m, v + m]: frac(v) >= m and
    // frac(v) + m < 1.  Fixed-point view (kFixMagic, |v| < 2^19): the low word lo = frac(v) 2^32 to within
    // 1/2 unit, so with mi = m 2^32 + 1/2 rounded up, lo in [mi, 2^32 - 1 - mi] for every pixel proves it
    // (the lane keeps min and max of lo: one v_min3 / v_max3 per two pixels).  The high word is
    // kFixHi + floor(v), and its low half floor(v) as a signed 16-bit value while |v| < 2^15, which
    // L1 < dec_l1_max guarantees (|v| <= Bmax L1 + m); v_sat_pk_u8_i16 then clamps two pixels to bytes
    // in one op.  A cube with a larger L1 (never from an encoder of 8-bit frames) goes to the replay.
    const double m = __builtin_fmin((double)l1_f * P.dec_G + P.dec_E, 0.5);
    const uint32_t mi = (uint32_t)__builtin_ceil(__fma_rn(m, 0x1p32, 0.5)) + 1u;  // + 1: m's own rounding
    bool flag = !(l1_f < P.dec_l1_max);
    uint32_t lo_min = 0xFFFFFFFFu, lo_max = 0u;
    uint32_t outw[D][NXC / 4];
#pragma unroll
    for (int z = 0; z < D; z++) {
#pragma unroll
        for (int wd = 0; wd < NXC / 4; wd++) {
            uint32_t hw[4];
#pragma unroll
            for (int e = 0; e < 4; e++) {
                const uint64_t fx = __builtin_bit_cast(uint64_t, cz[z][4 * wd + e]);  // w = v + kFixMagic
                hw[e] = (uint32_t)(fx >> 32);
                lo_min = min(lo_min, (uint32_t)fx);
                lo_max = max(lo_max, (uint32_t)fx);
            }
            // bytes 0..3 = clamp(floor(v_e), 0, 255): pairs of signed 16-bit floors, saturated to u8
            const uint32_t p01 = __builtin_amdgcn_perm(hw[1], hw[0], 0x05040100u);
            const uint32_t p23 = __builtin_amdgcn_perm(hw[3], hw[2], 0x05040100u);
            uint32_t w;
            asm("v_sat_pk_u8_i16_e32 %0, %1" : "=v"(w) : "v"(p01));
            asm("v_sat_pk_u8_i16_sdwa %0, %1 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD" : "+v"(w) : "v"(p23));
            asm volatile("" : "+v"(w));  // one output word at a time (bounded live range)
            outw[z][wd] = w;
        }
    }
    flag |= (lo_min < mi) | (lo_max > 0xFFFFFFFFu - mi);
    // ---- rare path: a lane with an uncertified pixel (a few per 2e9 pixels) has its 32 pixels replayed
    //      by the wave before the stores: the exact Java fold writes them to LDS and the lane takes its
    //      words from there (no second store of any address, no flag list, no fixup launch) ----
    const unsigned long long fl = __ballot(flag && valid);
    if (__builtin_expect(fl != 0ull, 0)) {
        uint32_t nrep = 0;
        for (unsigned long long rem = fl; rem != 0ull; rem &= rem - 1ull) {  // wave-uniform
            const int src = (int)__builtin_ctzll(rem);
            const int ci = (src >> 5) * (CPW / 2) + ((src & 15) / D);
            const uint8_t* ob = decode_replay_lane<D>(P.inv_coef_t, reload, wl, lane, cube0 + ci, src);
            if (lane == src) {
#pragma unroll
                for (int z = 0; z < D; z++)
#pragma unroll
                    for (int wd = 0; wd < NXC / 4; wd++) outw[z][wd] = *(const uint32_t*)(ob + z * NXC + 4 * wd);
            }
            wave_lds_sync();
            nrep += 32;
        }
        if (lane == 0 && P.replay_count) atomicAdd(P.replay_count + (blockIdx.x & (kCountSpread - 1)), nrep);
    }
    __builtin_amdgcn_s_setprio(2);  // the store phase ahead of the computing waves (as encode16_kernel)
    dec_store_tile<D, LOOP>(P, wl, lane, cube0, outw, valid);
}

// Block 0 zeroes the next call's counter slot, both halves (the two slots alternate between the
// encode and decode calls of a ctx; see EncodeParams)
__device__ __forceinline__ void dec_clear_next_slot(const DecodeParams& P) {
    if (blockIdx.x == 0 && P.replay_clear) {
#pragma unroll
        for (int i = 0; i < 2 * kCountSpread / kBlock; i++) P.replay_clear[i * kBlock + threadIdx.x] = 0u;
    }
}

template <int D, int PG>
__global__ __launch_bounds__(kBlock, 4) void decode_kernel(DecodeParams P) {
    __shared__ __attribute__((aligned(16))) char lds[kWavesPerBlock * kDecWaveLds];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    char* wl = lds + wave * kDecWaveLds;
    const uint32_t cube0 = (xcd_tile() * kWavesPerBlock + wave) * DecGeom<D>::CPW;
    int4 v[8];
    __builtin_amdgcn_s_setprio(3);  // a starting wave issues its loads ahead of the computing ones
    dec_load_tile<D>(P, cube0, lane, v);
    __builtin_amdgcn_s_setprio(0);
    dec_clear_next_slot(P);
    dec_stage_tile<D>(wl, lane, v);
    wave_lds_sync();
    decode_tile<D, PG>(P, wl, lane, cube0, [] {}, ReloadCubes<D>{P.in});
}

}  // namespace dct3d
