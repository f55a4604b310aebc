// dct3d_kernels.hip -- CDNA4 (gfx950) kernels of the 3D-DCT hot path (the device templates live in
// dct3d_encode_dev.h / dct3d_decode_dev.h; this file instantiates them, adds the fused Exp-Golomb
// kernels and the launchers).
//
// Work decomposition.  8x8x8 encode (encode16_kernel), decode, float drop-ins: 16 lanes per cube (2 D
// lanes at 8x8x4 decode), 32 values per lane, the permlane16 pair (l, l ^ 16) splitting each cube.
// 8x8x4 encode and the fused encode + Exp-Golomb: 8 lanes per cube, 8 cubes per wave ("row layout"
// lane (c, y) holds a[z][x]; "face layout" lane (c, kz[, h]) holds b[y][x]).  Layout changes are
// permlane16 swaps or a wave-private LDS transpose (no workgroup barrier: LDS ops of a wave execute in
// order); cube-major int32 / fp64 traffic is staged through the same region so that every global
// access of the wave is a contiguous 1 KiB (16 B per lane) burst.
//
// Encode (raster u8 -> quantised int32 cube-major), fp32, certified: rows -> S, m, A = max|x - m| ->
// pass X (exact integer front, centring folded into X0) -> pass Z -> pass Y -> q = v * fp32(1/step),
// n = rint(q), certified iff |q - n| < 0.5 - (A*G_s + E_s) (dct3d_plan.cpp).  DC = JavaRound(fp64(S) *
// coef_dc) exactly.  Open coefficients: 8x8x8 settles them in the wave (fp64 second certificate, then
// the exact Java fold); 8x8x4 folds them exactly in the wave, its 8 cubes in parallel (enc4_replay).
// Decode (quantised int32 cube-major -> raster u8), fp64, certified: staged loads -> fp64 dequantise +
// L1 -> inverse passes Y, X, Z (the last one adds the fixed-point offset) -> certificate on the low
// words, 16-bit floors saturated to bytes -> raster stores; uncertified cubes are replayed whole in the
// wave (exact Java InverseDCT fold) before the stores.
#include "dct3d_encode_dev.h"
#include "dct3d_decode_dev.h"

namespace dct3d {

// =============================================================================================
// Fused encode + Exp-Golomb, K1 (dct3d_encode_eg_dev; encoder.c:206-274 up to the deflate)
// =============================================================================================
// The wave's 8 cubes: rows -> transform -> quantise + certify exactly as encode_body, but the
// uncertified coefficients are recorded in a per-lane bit mask (bit ky*NB + x) and replayed by the
// wave itself (exact_coef) after the quantised cubes are staged in LDS as int16 (|q| <= 255*sqrt(cs)
// by Parseval, DC included).  Then lane (c', part) codes stream positions part*VPL .. part*VPL+VPL-1
// of cube c' (diagonal-slice order, CubeUtils.c:5-46; signed order-0 Exp-Golomb, ExpGolomb.c:32-64)
// into its own words of the segment's slot; eg_compact_kernel later concatenates the lanes.
// Signed order-0 Exp-Golomb (ExpGolomb.c:32-64): v <= 0 -> 1 - 2v, v > 0 -> 2v = max(2v, 1 - 2v); the
// code's width is 2 * bit_length(code) - 1.  K1 stages the codes, not the values: two per register
// through packed 16-bit ops (|v| <= 255*sqrt(512) < 2^13, so 2v and 1 - 2v fit int16).
typedef short eg_s16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t eg_code_pair(uint32_t hi, uint32_t lo) {
    const eg_s16x2 v = __builtin_bit_cast(eg_s16x2, __builtin_amdgcn_perm(hi, lo, 0x05040100u));
    const eg_s16x2 t = v + v;
    const eg_s16x2 c = __builtin_elementwise_max(t, (eg_s16x2)(1) - t);
    return __builtin_bit_cast(uint32_t, c);
}
// The code's width, 63 - 2*clz(code), as one v_mad_i32_i24 (the compiler would split it into a shift
// and an xor); code >= 1: a plain v_ffbh_u32
__device__ __forceinline__ uint32_t eg_width(uint32_t code) {
    uint32_t w;
    asm("v_mad_i32_i24 %0, %1, -2, 63" : "=v"(w) : "v"((uint32_t)__builtin_clz(code)));
    return w;
}
// g << w, then code OR-ed into the low word (a 32-bit OR: the code's upper bits are known zero there)
__device__ __forceinline__ uint64_t eg_push(uint64_t g, uint32_t w, uint32_t code) {
    const uint64_t t = g << (w & 63u);
    return ((uint64_t)(uint32_t)(t >> 32) << 32) | (uint32_t)((uint32_t)t | code);
}

// The same on a code held in 16-bit half H of a register (two codes per register): SDWA operand
// selects, so that the half is never unpacked (v_ffbh_u32 of the zero-extended half; v_or_b32 of it)
template <int H>
__device__ __forceinline__ uint32_t eg_width16(uint32_t x) {
    uint32_t z, w;
    if constexpr (H == 0)
        asm("v_ffbh_u32_sdwa %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_0" : "=v"(z) : "v"(x));
    else
        asm("v_ffbh_u32_sdwa %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1" : "=v"(z) : "v"(x));
    asm("v_mad_i32_i24 %0, %1, -2, 63" : "=v"(w) : "v"(z));
    return w;
}
template <int H>
__device__ __forceinline__ uint64_t eg_push16(uint64_t g, uint32_t w, uint32_t x) {
    const uint64_t t = g << (w & 63u);
    uint32_t lo;
    if constexpr (H == 0)
        asm("v_or_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0"
            : "=v"(lo) : "v"((uint32_t)t), "v"(x));
    else
        asm("v_or_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1"
            : "=v"(lo) : "v"((uint32_t)t), "v"(x));
    return ((uint64_t)(uint32_t)(t >> 32) << 32) | lo;
}

// Append W < 64 stream bits (the low W bits of g, MSB first) to a lane's pending bits (p: the low nb <
// 32 bits, nothing above them), branch-free.  The words completed (0, 1 or 2) go to the lane's next
// words of the segment through its buffer descriptor (a lane without a word stores out of range:
// dropped), except the lane's first word when it shares it with lane - 1 (dofs == hofs): that one is
// kept in `head` for lane - 1's last store.  The bits left pending are the low T mod 32 bits of
// p * 2^W + g.
__device__ __forceinline__ void eg_append(uint64_t g, uint32_t W, uint32_t& p, uint32_t& nb,
                                          __amdgpu_buffer_rsrc_t seg, uint32_t& dofs, uint32_t hofs,
                                          uint32_t& head) {
    const uint32_t T = nb + W;
    const uint32_t w0 = (p << ((32u - nb) & 31u)) | (uint32_t)(g >> ((T - 32u) & 63u));
    const uint32_t w1 = (uint32_t)(g >> ((T - 64u) & 63u));
    const bool hd = dofs == hofs;
    __builtin_amdgcn_raw_buffer_store_b32(w0, seg, (int)(T >= 32u && !hd ? dofs : 0x80000000u), 0, 0);
    __builtin_amdgcn_raw_buffer_store_b32(w1, seg, (int)(T >= 64u ? dofs + 4u : 0x80000000u), 0, 0);
    head = T >= 32u && hd ? w0 : head;
    dofs += (T >> 5) << 2;
    p = __builtin_amdgcn_ubfe((uint32_t)((uint64_t)p << W) | (uint32_t)g, 0u, T & 31u);
    nb = T & 31u;
}

// The lane's VPL codes (cds: two per register, lane order = stream order within the segment) into the
// segment's slot.  First the lane's bit count (the sum of its code widths, 63 - 2 clz each: zs = the sum of
// the leading-zero counts), the wave's exclusive scan of the counts: the lane's first bit in the segment.
// Then the codes: 8 concatenated into one 64-bit group when they fit (W < 64; else one by one), each group
// appended to the lane's pending bits -- which start as the off mod 32 bits of the lanes before it, zeros
// here -- with at most two words out, at the segment's word index: the slot holds the segment's stream,
// and eg_compact_kernel only shifts it to the segment's offset.  A word two lanes share (every coding lane
// has >= VPL bits, so at most two) is stored once, by the first lane, merged with the second lane's part
// through a shuffle.  (Round 4 before: lane-local words in slot columns, concatenated by the compaction:
// 0.55 GB of partial-line slot stores and a lane bit-count array for a 0.37 GB stream.  Buffering the
// words in LDS needs the values in registers to free the region: +6 % kernel time for the pack / unpack.)
template <int VPL>
__device__ __forceinline__ void eg_lane_emit(const EgFusedParams& E, const uint32_t (&cds)[VPL / 2], uint32_t zs,
                                             bool lvalid, int lane, uint32_t wid) {
    const uint32_t lbits = lvalid ? 63u * VPL - 2u * zs : 0u;
    uint32_t incl = lbits;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(incl, o, 64);
        if (lane >= o) incl += t;
    }
    const uint32_t off = incl - lbits;  // the lane's first bit in the segment
    // the segment's slot (wave-uniform base and size) as a buffer descriptor; each store adds a 32-bit
    // lane offset
    const __amdgpu_buffer_rsrc_t seg = __builtin_amdgcn_make_buffer_rsrc(
        E.slot + (size_t)__builtin_amdgcn_readfirstlane(wid) * E.seg_cap, (short)0, (int)(E.seg_cap * 4u), 0x00020000);
    uint32_t dofs = (off >> 5) * 4u;  // byte offset of the lane's next word in the segment
    const uint32_t hofs = (off & 31u) ? dofs : 0xFFFFFFFFu;  // its first word, when shared with lane - 1
    uint32_t p = 0, nb = lvalid ? (off & 31u) : 0u, head = 0;
    if (lvalid) {
#pragma unroll
        for (int i0 = 0; i0 < VPL; i0 += 8) {
            uint32_t cd[8], w[8];
#pragma unroll
            for (int e = 0; e < 8; e++) cd[e] = (e & 1) ? cds[(i0 + e) / 2] >> 16 : cds[(i0 + e) / 2] & 0xFFFFu;
            // group 0 (the DC and the lowest frequencies: > 64 bits in every wave of 1080p ramp and uniform
            // content, <= 64 bits per half in all of them) as two halves of 4 codes; the others as one
            // group of 8 (> 64 bits in 2 % of the waves at group 1 on uniform content, never later)
            constexpr int NH = 2;
            uint64_t g[NH] = {0, 0};
            uint32_t W[NH] = {0, 0};
#pragma unroll
            for (int e = 0; e < 8; e++) {
                const uint32_t x = cds[(i0 + e) / 2];
                w[e] = (e & 1) ? eg_width16<1>(x) : eg_width16<0>(x);
                const int h = i0 == 0 ? e / 4 : 0;
                g[h] = (e & 1) ? eg_push16<1>(g[h], w[e], x) : eg_push16<0>(g[h], w[e], x);
                W[h] += w[e];
            }
            if (__builtin_expect(W[0] < 64u && W[1] < 64u, 1)) {
                eg_append(g[0], W[0], p, nb, seg, dofs, hofs, head);
                if (i0 == 0) eg_append(g[1], W[1], p, nb, seg, dofs, hofs, head);
            } else {
#pragma unroll
                for (int e = 0; e < 8; e++) eg_append(cd[e], w[e], p, nb, seg, dofs, hofs, head);
            }
        }
    }
    // the lane's last, partial word, completed by lane + 1's first bits (lane + 1 starts inside it)
    const uint32_t nh = __shfl_down(head, 1, 64);
    __builtin_amdgcn_raw_buffer_store_b32((p << ((32u - nb) & 31u)) | (lane < 63 ? nh : 0u), seg,
                                          (int)(nb ? dofs : 0x80000000u), 0, 0);
    if (lane == 63) E.seg_bits[wid] = incl;
}

// Byte offset of cube-major code k (k = (kz*8 + ky)*8 + kx) in K1's staging of one cube.  8x8x8: the rows
// of face kz are rotated by kz (row ky at slot (ky + kz) mod 8), so that the 16-byte row stores of a
// ds_write_b128 lane group -- one cube's 8 faces, the same ky -- land on 8 different 4-bank groups (round 6:
// unrotated, all 8 sat on one: 7 extra LDS cycles per group, 56 per store instruction, most of K1's
// SQ_LDS_BANK_CONFLICT); the emission's scattered reads are unchanged on average (3.25 -> 3.31 extra cycles
// per read, tools/k1_lds_sim.py).
template <int D>
__device__ __forceinline__ uint32_t k1_code_off(uint32_t k) {
    if constexpr (D == 8) return (k >> 6) * 128u + ((((k >> 3) + (k >> 6)) & 7u) << 4) + (k & 7u) * 2u;
    else return (k >> 6) * 128u + (k & 63u) * 2u;
}

template <int D>
__global__ __launch_bounds__(kBlock, 4) void encode_eg_kernel(EncodeParams P, EgFusedParams E) {
    constexpr int CS = 64 * D;
    constexpr int NB = (D == 8) ? 8 : 4;
    constexpr int NI = 7 + NB;
    constexpr int VPL = CS / 8;            // stream values per lane
    // uint16 cube-major staging: face kz at kz * FACE (a multiple of 16: the rows go as 16-byte stores), cube
    // at c * CUBE_B.  8x8x8: cubes 1,056 B apart (a host search over the strides within the wave's region: the
    // emission's scattered 16-bit reads 2.9 -> 2.6 LDS cycles; before: 1,040); 8x8x4: 528 B
    constexpr int FACE = 128;
    static_assert(FACE == 128, "k1_code_off's face stride");
    constexpr int CUBE_B = (D == 8) ? 1056 : 2 * CS + 16;
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
    // the rows in flight first, issued at the top priority (as encode16_kernel's: under oldest-first issue
    // they queue behind the computing waves' VALU work; c7 -0.4 %, profiles/r05/c7_ab/7_prio)
    __builtin_amdgcn_s_setprio(3);
    load_rows<D>(P, cube0 + (lane >> 3), cube0 + (lane >> 3) < P.n_cubes, lane & 7, raw);
    __builtin_amdgcn_s_setprio(0);
    {  // both loads in flight before the LDS writes (a strided loop waited one round trip per pass)
        static_assert(CS % kBlock == 0, "whole passes");
        uint16_t t[CS / kBlock];
#pragma unroll
        for (int r = 0; r < CS / kBlock; r++) t[r] = E.diag[threadIdx.x + r * kBlock];
#pragma unroll
        for (int r = 0; r < CS / kBlock; r++) s_pos[threadIdx.x + r * kBlock] = (uint16_t)k1_code_off<D>(t[r]);
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

    // stage the cubes' Exp-Golomb codes as uint16, cube-major (k = (kz*8 + ky)*8 + kx at byte 2k of cube c)
#pragma unroll
    for (int ky = 0; ky < 8; ky++) {
        char* row = wl + c * CUBE_B + kz * FACE + ((D == 8) ? (((ky + kz) & 7) << 4) : 2 * (ky * 8 + kx0));
        if constexpr (D == 8) {
            *(uint4*)row = make_uint4(eg_code_pair(qv[ky][1], qv[ky][0]), eg_code_pair(qv[ky][3], qv[ky][2]),
                                      eg_code_pair(qv[ky][5], qv[ky][4]), eg_code_pair(qv[ky][7], qv[ky][6]));
        } else {
            *(uint2*)row = make_uint2(eg_code_pair(qv[ky][1], qv[ky][0]), eg_code_pair(qv[ky][3], qv[ky][2]));
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
            if (lane == 0) *(uint16_t*)(wl + sc * CUBE_B + k1_code_off<D>(k)) = (uint16_t)(q > 0 ? 2 * q : 1 - 2 * q);
            if (lane == src) {
                if (fm_lo) fm_lo &= fm_lo - 1;
                else fm_hi &= fm_hi - 1;
            }
            wave_lds_sync();
        }
    }

#if defined(DCT3D_K1_SPLIT) && DCT3D_K1_SPLIT == 1  // DIAGNOSTIC timing split only: transform, staging, replays
    if (lane == 0) E.seg_bits[wid] = 256u;  // a whole, in-bounds segment for the scan, compaction and stitch
    return;
#endif
    // Exp-Golomb: lane (cp, part) codes stream positions part*VPL .. +VPL-1 of cube cp (lane order =
    // stream order), read from the staged codes 8 at a time (eg_lane_emit)
    const int cp = lane >> 3, part = lane & 7;
    const bool lvalid = cube0 + cp < P.n_cubes;
    const char* cb = wl + cp * CUBE_B;
    uint32_t zs = 0;  // sum of the leading-zero counts of the lane's codes
    uint32_t cds[VPL / 2];  // the lane's codes, two per register, kept for the emission
    if (lvalid) {
#pragma unroll
        for (int i0 = 0; i0 < VPL; i0 += 8) {
            const uint4 pp = *(const uint4*)&s_pos[part * VPL + i0];
            const uint32_t pw[4] = {pp.x, pp.y, pp.z, pp.w};
#pragma unroll
            for (int e = 0; e < 8; e += 2) {
                const uint32_t lo = *(const uint16_t*)(cb + (pw[e >> 1] & 0xFFFFu));
                const uint32_t hi = *(const uint16_t*)(cb + (pw[e >> 1] >> 16));
                cds[(i0 + e) / 2] = lo | (hi << 16);
                zs += __builtin_clz(lo) + __builtin_clz(hi);
            }
        }
    }
#if defined(DCT3D_K1_SPLIT) && DCT3D_K1_SPLIT == 2  // DIAGNOSTIC timing split only: + the codes and widths
    asm volatile("" ::"v"(zs));
#pragma unroll
    for (int i = 0; i < VPL / 2; i++) asm volatile("" ::"v"(cds[i]));
    if (lane == 0) E.seg_bits[wid] = 256u;
    return;
#endif
    eg_lane_emit<VPL>(E, cds, zs, lvalid, lane, wid);
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
    const uint32_t cube0 = (xcd_tile() * kWavesPerBlock + wave) * CPW;
    if (cube0 >= n_cubes) return;  // wave-uniform
    {
        int4 v[8];
        __builtin_amdgcn_s_setprio(3);
        dec_load_tile_p<D>((const char*)in, n_cubes, cube0, lane, v);
        __builtin_amdgcn_s_setprio(0);
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
            for (int e = 0; e < NXC; e += 4) {  // non-temporal: whole 128-byte lines, written once
                typedef float f32x4_t __attribute__((ext_vector_type(4)));
                __builtin_nontemporal_store(f32x4_t{v[e], v[e + 1], v[e + 2], v[e + 3]}, (f32x4_t*)(o + z * 64 + e));
            }
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
// The rare exact replay re-parses its cube from the stream at the cube's marks (lanes 0 .. CS/32 - 1,
// 32 values each, global reads: the wave's window is gone by then).
template <int D>
struct ReloadStream {
    const uint32_t* words;
    uint64_t n_words;
    const uint16_t* mark;
    const uint64_t* mark_base;
    const uint16_t* diag;  // the block's LDS copy
    __device__ __forceinline__ void operator()(uint32_t g, double* cf, int lane) const {
        constexpr int PARTS = 64 * D / 32;
        if (lane < PARTS) {
            BitReader<GlobalBits> r{GlobalBits{words, n_words}, 0, 0, 0, 0};
            r.seek(mark_serial(mark, mark_base, (uint64_t)g * PARTS + lane));
            for (int i = 0; i < 32; i++) {
                uint32_t code = 1u;
                (void)r.get(code);
                const int k = diag[lane * 32 + i];
                const int kz = k / 64, ky = (k / 8) & 7, kx = k & 7;
                cf[k] = (double)eg_value(code) * (double)max(1, 5 * (kx + ky + kz));
            }
        }
    }
};

// lane 0's 64-bit value in scalar registers (readfirstlane returns int: widened from uint32_t, unsigned)
__device__ __forceinline__ uint64_t uniform_u64(uint64_t x) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)x);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(x >> 32));
    return ((uint64_t)hi << 32) | lo;
}

// NG groups per wave (a group = the wave's CPW cubes = 64 marks), the block's 4 waves on 4 consecutive
// groups per round (dec_store_tile's block stores).  The next group's marks are loaded while this
// group's window is parsed, and its window words (NWP per lane, as far as they reach) while this group
// is transformed, so the mark -> window -> parse chain of global round trips is paid once per wave, not
// once per group.  Carried across the transform: the NWP words, the lane's mark relative to the window
// (32 bits) and two wave-uniform 64-bit values (scalar registers).  NG = 1: no look-ahead.
template <int D, int NG>
__global__ __launch_bounds__(kBlock, 4) void decode_eg_kernel(DecodeParams P, EgDecParams E) {
    using G = DecGeom<D>;
    constexpr uint32_t CS = G::CS, PARTS = CS / 32, CPW = G::CPW;
    static_assert(CPW * CS == 2048 && PARTS * CPW == 64, "one wave = 64 marks");
    constexpr uint32_t WIN = kDecWaveLds / 4 - 1;  // 2,319 words >= 2,048 values x 27 bits (+ win[-1])
    constexpr int NWP = 4;                     // window words per lane loaded ahead (256: 4 bits per value)
    __shared__ __attribute__((aligned(16))) char lds[kWavesPerBlock * kDecWaveLds];
    __shared__ uint16_t s_diag[CS];
    // staging byte offset (within a cube) of stream position part * 32 + j at s_soff[part * SOFF + j]:
    // rows of 40 entries (80 B), so that the 16 parts' 16-byte reads fall on distinct banks
    constexpr uint32_t SOFF = 40;
    __shared__ __attribute__((aligned(16))) uint16_t s_soff[PARTS * SOFF];
    dec_clear_next_slot(P);
    if (blockIdx.x == 0 && threadIdx.x == 0 && E.status_host) {  // the verdict to the host: the words, the tag
        uint64_t w[6];
#pragma unroll
        for (int i = 0; i < 6; i++) E.status_host[i] = w[i] = E.status[i];
        const uint32_t fl = (uint32_t)(w[2] & 7u) | (w[4] < E.n_values ? 8u : 0u);  // flags, short by the scan
        __hip_atomic_store(E.status_host + 6, hand_off_tag(E.seq, w[1], fl), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (blockIdx.x == 0 && threadIdx.x < 6 && E.status_clear) E.status_clear[threadIdx.x] = 0u;
    // corrupt / short / empty stream: reported by the mark pass (block-uniform)
    if (E.status[2] != 0 || E.n_words == 0) return;
    const bool long_codes = E.status[3] != 0;  // the stream holds a code of 33+ bits (the mark pass)
    {  // both loads in flight before the LDS writes
        static_assert(CS % kBlock == 0, "whole passes");
        uint16_t t[CS / kBlock];
#pragma unroll
        for (uint32_t r = 0; r < CS / kBlock; r++) t[r] = E.diag[threadIdx.x + r * kBlock];
#pragma unroll
        for (uint32_t r = 0; r < CS / kBlock; r++) {
            const uint32_t i = threadIdx.x + r * kBlock, k = t[r];
            s_diag[i] = t[r];
            s_soff[(i / 32) * SOFF + i % 32] = (uint16_t)((k >> 6) * G::SA_F + (k & 63) * 4);
        }
    }
    __syncthreads();
    const int lane0 = threadIdx.x & 63, wave = threadIdx.x >> 6;
    char* wl = lds + wave * kDecWaveLds;
    uint32_t* win = (uint32_t*)wl + 1;  // the window one word into the region: parse_step reads win[-1]
    const uint64_t n_marks = E.n_values / 32;
    const uint32_t row0 = xcd_tile() * NG;  // the block's first round of 4 groups
    auto cube_of = [&](int i) { return P.cube_base + ((row0 + (uint32_t)i) * kWavesPerBlock + wave) * CPW; };
    // the group's marks as loaded: its first (a whole position), the lane's low 16 bits (value 32 * (m0 +
    // lane); a lane past the last mark: ~0u) and the end of its bit range (all lanes alike).  They
    // are combined in open_window, after the parse they are loaded across (combined here, the wait for them
    // sat before the parse)
    static_assert(kMarkGroup == 64, "a group = one mark group");
    auto load_marks = [&](int lane, uint32_t cube0, uint64_t& gb, uint32_t& myl, uint64_t& last) {
        const uint64_t m0 = (uint64_t)cube0 * CS / 32;
        // a wave past the last group (or the look-ahead of the group after it) reads no mark_base entry:
        // it holds n_marks / kMarkGroup + 1 of them
        gb = m0 < n_marks ? E.mark_base[m0 / kMarkGroup] : 0u;
        myl = m0 + lane < n_marks ? (uint32_t)E.mark[m0 + lane] : ~0u;
        last = m0 + 64 < n_marks ? E.mark_base[m0 / kMarkGroup + 1] : E.status[1];
    };
    // window of a group: first word w0 (the first mark's), the lane's mark relative to bit 32 w0, the
    // words up to the end mark (+5 slack: parse_win); its first NWP * 64 words requested (clamped into the stream)
    auto open_window = [&](int lane, uint64_t gb, uint32_t myl, uint64_t last, uint64_t& w0, uint32_t& rel,
                           uint64_t& span, uint32_t (&t)[NWP]) {
        w0 = uniform_u64(gb >> 5);  // the group's first mark
        // relative to bit 32 w0: the mark's offset from the group's first, + gb % 32; a lane past the last
        // mark (the unused cubes of a partial last group) parses from the window's first bit, inside the window
        const uint32_t off = mark_offset(myl, (uint16_t)gb);
        rel = myl <= 0xFFFFu ? (uint32_t)(gb & 31) + off : 0u;
        const uint64_t lw = uniform_u64(last);
        span = (lw >> 5) + 5 - w0;
        // word w0 + j from a scalar base, j clamped into the stream in 32 bits (a look-ahead past the last
        // group reads a w0 made of other data: clamped too)
        const uint64_t wb = min(w0, E.n_words - 1);
        const uint32_t jmax = (uint32_t)min(E.n_words - 1 - wb, (uint64_t)0xFFFFFFFFu);
#pragma unroll
        for (int b = 0; b < NWP; b++) t[b] = E.words[wb + min((uint32_t)(b * 64 + lane), jmax)];
    };
    uint64_t w0, span;
    uint32_t rel;
    uint32_t pw[NWP];
    {
        uint64_t gb, last;
        uint32_t myl;
        __builtin_amdgcn_s_setprio(3);  // marks and window loads ahead of the computing waves
        load_marks(lane0, cube_of(0), gb, myl, last);
        open_window(lane0, gb, myl, last, w0, rel, span, pw);
        __builtin_amdgcn_s_setprio(0);
    }
    for (int i = 0; i < NG; i++) {
        const uint32_t cube0 = cube_of(i);
        if (cube0 >= P.n_cubes) break;  // wave-uniform; every later group of the wave is past the end too
        // the lane's addresses and constants are made inside each round, not hoisted and held across
        // the transform (which needs the registers)
        int lane = lane0;
        asm volatile("" : "+v"(lane));
        const bool fits = span <= WIN;  // wave-uniform; else the parse reads global memory (parse_codes)
        const uint32_t nwin = (uint32_t)(fits ? span : 0);
        // Everything before the group's transform runs at priority 2 (the look-ahead loads at 3): the window
        // staging, the parse (a chain of dependent LDS reads) and the scatter, so that a wave in these
        // latency-bound phases issues ahead of the other waves' transform VALU work instead of queueing
        // behind it under oldest-first issue, and the transform fills the gaps.  Consumer 2,466 -> 2,375 us
        // (the parse alone) -> 2,275 us per c8 step, A/B x 3 on one box each (profiles/r05/consumer/parse_prio).
        __builtin_amdgcn_s_setprio(2);
        // window words past the stream's end read as zero (w0 < n_words: the group's first mark is in it)
        const uint32_t nlive = (uint32_t)min((uint64_t)nwin, E.n_words - w0);
        // the look-ahead words, in rows of 64 (a wave-uniform test per row, no per-lane branch: the region
        // holds NWP * 64 words, and those past the window are never read)
        static_assert(NWP * 64 <= WIN, "look-ahead inside the region");
#pragma unroll
        for (int b = 0; b < NWP; b++) {
            const uint32_t j = b * 64 + lane;
            if (b * 64 < nwin) win[j] = j < nlive ? __builtin_bswap32(pw[b]) : 0u;
        }
        // the rest of a window longer than the look-ahead (content above 4 bits per value): 4 words per
        // lane per round, all loads issued before the first LDS write
        for (uint32_t i0 = NWP * 64; i0 < nwin; i0 += 256) {
            uint32_t t[4];
#pragma unroll
            for (int b = 0; b < 4; b++) t[b] = E.words[min(w0 + i0 + b * 64 + lane, E.n_words - 1)];
#pragma unroll
            for (int b = 0; b < 4; b++) {
                const uint32_t j = i0 + b * 64 + lane;
                if (j < nwin) win[j] = j < nlive ? __builtin_bswap32(t[b]) : 0u;
            }
        }
        uint64_t gb_n = 0, last_n = 0;
        uint32_t myl_n = 0;
        // the look-ahead loads at the top priority (as the first group's): issued ahead of the other waves'
        // parse and transform work, not behind it (consumer 2,520 -> 2,454 us per c8 step,
        // profiles/r05/consumer/prio)
        __builtin_amdgcn_s_setprio(3);
        if (i + 1 < NG) load_marks(lane, cube_of(i + 1), gb_n, myl_n, last_n);  // in flight during the parse
        __builtin_amdgcn_s_setprio(2);
        wave_lds_sync();
        uint32_t v[32];  // codes: decode_tile<CODES> converts them in its dequantisation
        parse_codes<32>(E, win, nwin, w0, fits, long_codes, rel, v);
        __builtin_amdgcn_s_setprio(3);
        if (i + 1 < NG) open_window(lane, gb_n, myl_n, last_n, w0, rel, span, pw);  // in flight during the transform
        __builtin_amdgcn_s_setprio(2);
        wave_lds_sync();
        {  // each value to its diagonal position in the staging: 8 offsets per 16-byte table read
            const uint32_t c = lane / PARTS, part = lane % PARTS;
            char* cb = wl + c * G::SA_C;
            const uint4* so = (const uint4*)(s_soff + part * SOFF);
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const uint4 o = so[q];
                const uint32_t w[4] = {o.x, o.y, o.z, o.w};
#pragma unroll
                for (int e = 0; e < 8; e++)
                    *(uint32_t*)(cb + ((w[e >> 1] >> (16 * (e & 1))) & 0xFFFFu)) = v[q * 8 + e];
            }
        }
        wave_lds_sync();
        __builtin_amdgcn_s_setprio(0);  // the transform
        decode_tile<D, 1, (NG > 1), true>(P, wl, lane, cube0, [] {}, ReloadStream<D>{E.words, E.n_words, E.mark, E.mark_base, s_diag});
        // the region receives the next group's window: after a block store (its rows are read by every
        // wave of the block) the whole block must be past it (block-uniform condition, as dec_store_tile's)
        if (i + 1 < NG) {
            if (P.blk_store && cube0 - (uint32_t)wave * CPW + kWavesPerBlock * CPW <= P.n_cubes) __syncthreads();
            else wave_lds_sync();
        }
    }
}

// =============================================================================================
// Launchers
// =============================================================================================
// Encode: 8x8x8 = encode16_kernel (16 lanes per cube, in-wave exact replay, one launch per call);
// 8x8x4 = encode_kernel<4> (8 lanes per cube, in-wave exact replay, one launch).  Both store the int32
// output non-temporally.  The variants that lost (8 lanes per cube at 8x8x8, plain stores, NT loads,
// LDS-padded occupancy) are recorded in profiles/r01/encode_variant_sweep.txt, not built.
namespace {
template <int D>
void launch_enc_eg_t(const EncodeParams& P, const EgFusedParams& E, hipStream_t st) {
    const uint32_t groups = (P.n_cubes + kCubesPerWave - 1) / kCubesPerWave;
    const uint32_t blocks = (groups + kWavesPerBlock - 1) / kWavesPerBlock;
    hipLaunchKernelGGL((encode_eg_kernel<D>), dim3(blocks), dim3(kBlock), 0, st, P, E);
}
}  // namespace

int launch_encode(int D, const EncodeParams& P, hipStream_t st) {
    if (P.n_cubes == 0) return 0;
    if (D == 8) {
        const uint32_t groups = (P.n_cubes - P.g_base + kE16CPW - 1) / kE16CPW;
        const uint32_t blocks = (groups + kWavesPerBlock - 1) / kWavesPerBlock;
        hipLaunchKernelGGL((encode16_kernel<true, 0>), dim3(blocks), dim3(kBlock), 0, st, P);
    } else {
        const uint32_t groups = (P.n_cubes - P.g_base + kCubesPerWave - 1) / kCubesPerWave;
        const uint32_t blocks = (groups + kWavesPerBlock - 1) / kWavesPerBlock;
        hipLaunchKernelGGL((encode_kernel<4, true>), dim3(blocks), dim3(kBlock), 0, st, P);
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_encode_eg(int D, const EncodeParams& P, const EgFusedParams& E, hipStream_t st) {
    if (P.n_cubes == 0) return 0;
    if (D == 8) launch_enc_eg_t<8>(P, E, st);
    else launch_enc_eg_t<4>(P, E, st);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// One butterfly per pin group (pin groups 1 / 2 / 4 / none measured within 1 %; non-temporal dword
// output stores were 26 % slower: profiles/r01/decode_variant_sweep.txt).
int launch_decode(int D, const DecodeParams& P, hipStream_t st) {
    if (P.n_cubes == 0) return 0;
    const uint32_t per = (D == 8 ? DecGeom<8>::CPW : DecGeom<4>::CPW) * kWavesPerBlock;
    const uint32_t groups = (uint32_t)((P.n_cubes + per - 1) / per);
    if (D == 8) hipLaunchKernelGGL((decode_kernel<8, 1>), dim3(groups), dim3(kBlock), 0, st, P);
    else hipLaunchKernelGGL((decode_kernel<4, 1>), dim3(groups), dim3(kBlock), 0, st, P);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

namespace {
template <int D, int NG>
void launch_dec_eg_t(const DecodeParams& P, const EgDecParams& E, hipStream_t st) {
    constexpr uint32_t cpw = DecGeom<D>::CPW;
    const uint32_t groups = (P.n_cubes - P.cube_base + cpw - 1) / cpw;  // cube_base: a multiple of cpw
    const uint32_t blocks = (groups + kWavesPerBlock * NG - 1) / (kWavesPerBlock * NG);
    hipLaunchKernelGGL((decode_eg_kernel<D, NG>), dim3(blocks), dim3(kBlock), 0, st, P, E);
}
template <int D>
void launch_dec_eg_d(const DecodeParams& P, const EgDecParams& E, int ng, hipStream_t st) {
    switch (ng) {
        case 1: launch_dec_eg_t<D, 1>(P, E, st); break;
        case 2: launch_dec_eg_t<D, 2>(P, E, st); break;
        case 4: launch_dec_eg_t<D, 4>(P, E, st); break;
        default: launch_dec_eg_t<D, 8>(P, E, st); break;
    }
}
}  // namespace

int launch_decode_eg(int D, const DecodeParams& P, const EgDecParams& E, int groups_per_wave, hipStream_t st) {
    if (P.n_cubes == 0) return 0;
    if (D == 8) launch_dec_eg_d<8>(P, E, groups_per_wave, st);
    else launch_dec_eg_d<4>(P, E, groups_per_wave, st);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}


}  // namespace dct3d
