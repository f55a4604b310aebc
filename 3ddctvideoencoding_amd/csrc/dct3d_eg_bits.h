// dct3d_eg_bits.h -- Exp-Golomb bit reading on the device, shared by the stream decoder
// (dct3d_eg.hip) and the fused stream -> raster decode (dct3d_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "dct3d_kernels.h"

namespace dct3d {

// stream words [w0, w0 + n), byte-swapped to MSB-first, in LDS; zero outside (past the end of the
// data -- and, on a corrupt stream only, past the window)
struct LdsBits {
    const uint32_t* s;
    uint64_t w0;
    uint32_t n;
    __device__ __forceinline__ uint32_t word(uint64_t k) const {
        const uint64_t i = k - w0;
        const uint32_t v = s[i < n ? i : 0];  // unconditional read (a read under a branch is waited at the join)
        return i < n ? v : 0u;
    }
};
// the stream in global memory (the fused decode's re-parse of a replayed cube: rare, latency-bound)
struct GlobalBits {
    const uint32_t* w;
    uint64_t nw;
    __device__ __forceinline__ uint32_t word(uint64_t k) const {
        const uint32_t v = w[k < nw ? k : nw - 1];
        return k < nw ? __builtin_bswap32(v) : 0u;
    }
};
__device__ __forceinline__ uint32_t stream_word(const EgDecParams& P, uint64_t k) {
    return k < P.n_words ? __builtin_bswap32(P.words[k]) : 0u;
}

template <class Src>
struct BitReader {
    Src L;
    uint64_t next;   // index of the word held in `pre`
    uint64_t buf;    // left-aligned bits [pos, pos + avail)
    int avail;
    uint64_t pos;
    uint32_t pre;    // word `next`, read one refill ahead: some lane of the wave refills on almost every
                     // code, so a read on demand put its full latency on every code
    __device__ __forceinline__ void seek(uint64_t p) {
        pos = p;
        const uint64_t k = p >> 5;
        const int sh = (int)(p & 31);
        buf = (((uint64_t)L.word(k) << 32) | L.word(k + 1)) << sh;
        avail = 64 - sh;
        next = k + 2;
        pre = L.word(next);
    }
    __device__ __forceinline__ void refill() {
        if (avail <= 32) {
            buf |= (uint64_t)pre << (32 - avail);
            avail += 32;
            pre = L.word(++next);
        }
    }
    // A run of 1-bit codes (value 0, the common case: ~80 % of the codes of quantised content):
    // consumes up to maxn of them at once (clz of the complement); returns how many.  The run stops at
    // a 0 bit (a longer code starts), at maxn, or where the buffered bits end (call again).
    __device__ __forceinline__ uint32_t ones(uint32_t maxn) {
        refill();
        const uint64_t inv = ~buf;
        uint32_t n1 = inv ? (uint32_t)__clzll((long long)inv) : 64u;
        n1 = min(min(n1, (uint32_t)avail), maxn);
        buf = n1 >= 64 ? 0ull : buf << n1;
        avail -= (int)n1;
        pos += n1;
        return n1;
    }
    // the next buffered bit is 0 (a code longer than one bit starts here)
    __device__ __forceinline__ bool at_long_code() const { return avail > 0 && !(buf >> 63); }
    // one codeword: false when 32 zero bits come first (invalid); *code = the (z+1)-bit value
    __device__ __forceinline__ bool get(uint32_t& code) {
        refill();
        const int z = __clz((int)(uint32_t)(buf >> 32));  // 32: the top 32 bits are zero (invalid)
        if (z >= 32) return false;
        const int width = 2 * z + 1;
        if (width <= avail) {
            code = (uint32_t)(buf >> (64 - width));
            buf <<= width;
            avail -= width;
            pos += (uint64_t)width;
        } else {  // a long code straddling the buffer: read it at its absolute position
            const uint64_t k = pos >> 5;
            const int sh = (int)(pos & 31);
            const uint64_t hi = (((uint64_t)L.word(k) << 32) | L.word(k + 1)) << sh;
            const uint64_t win = sh ? (hi | ((uint64_t)L.word(k + 2) >> (32 - sh))) : hi;
            code = (uint32_t)(win >> (64 - width));
            seek(pos + (uint64_t)width);
        }
        return true;
    }
};

// The same reader over an LDS window with window-relative 32-bit positions (a window holds < 2^18
// bits): the per-code 64-bit index, compare and carry arithmetic of absolute positions was most of the
// parse's instructions.  Word i of the window is s[i] (i < n), zero beyond.
struct WinReader {
    const uint32_t* s;
    uint32_t n;
    uint32_t next;   // index of the word held in `pre`
    uint64_t buf;    // left-aligned bits [pos, pos + avail)
    int avail;
    uint32_t pos;
    uint32_t pre;    // word `next` as read: zeroed past the window only where it is used, so that the
                     // LDS read's wait falls at the next refill, not right behind the read
    __device__ __forceinline__ uint32_t word(uint32_t i) const {
        const uint32_t v = s[i < n ? i : 0u];  // unconditional read
        return i < n ? v : 0u;
    }
    __device__ __forceinline__ void seek(uint32_t p) {
        pos = p;
        const uint32_t k = p >> 5;
        const int sh = (int)(p & 31);
        buf = (((uint64_t)word(k) << 32) | word(k + 1)) << sh;
        avail = 64 - sh;
        next = k + 2;
        pre = s[next < n ? next : 0u];
    }
    __device__ __forceinline__ void refill() {
        if (avail <= 32) {
            buf |= (uint64_t)(next < n ? pre : 0u) << (32 - avail);
            avail += 32;
            ++next;
            pre = s[next < n ? next : 0u];
        }
    }
    __device__ __forceinline__ uint32_t ones(uint32_t maxn) {
        refill();
        const uint64_t inv = ~buf;
        uint32_t n1 = inv ? (uint32_t)__clzll((long long)inv) : 64u;
        n1 = min(min(n1, (uint32_t)avail), maxn);
        buf = n1 >= 64 ? 0ull : buf << n1;
        avail -= (int)n1;
        pos += n1;
        return n1;
    }
    __device__ __forceinline__ bool at_long_code() const { return avail > 0 && !(buf >> 63); }
    __device__ __forceinline__ bool get(uint32_t& code) {
        refill();
        const uint32_t hi32 = (uint32_t)(buf >> 32);
        if (hi32 == 0u) return false;  // 32 zero bits: invalid
        const int width = 2 * __builtin_clz(hi32) + 1;
        const bool fits = width <= avail;
        // the common case without a divergent if / else
        code = (uint32_t)(buf >> (64 - width));
        buf <<= width;
        avail -= width;
        pos += (uint32_t)width;
        if (__builtin_expect(__ballot(!fits) != 0ull, 0)) {
            if (!fits) {  // a long code straddling the buffer (|v| >= 2^16: never for quantised 8-bit content)
                const uint32_t p = pos - (uint32_t)width;
                const uint32_t k = p >> 5;
                const int sh = (int)(p & 31);
                const uint64_t hi = (((uint64_t)word(k) << 32) | word(k + 1)) << sh;
                const uint64_t w = sh ? (hi | ((uint64_t)word(k + 2) >> (32 - sh))) : hi;
                code = (uint32_t)(w >> (64 - width));
                seek(pos);
            }
        }
        return true;
    }
};

// signed value of a code (ExpGolombReader.java:52-62, as eg_value): code = 2v (v > 0) or 1 - 2v
// (v <= 0), i.e. v = code >> 1, negated when the code is odd
__device__ __forceinline__ int32_t eg_value_fast(uint32_t code) {
    const int32_t m = -(int32_t)(code & 1u);
    return ((int32_t)(code >> 1) ^ m) - m;
}

__device__ __forceinline__ int32_t eg_value(uint32_t code) {  // ExpGolombReader.java:52-62
    const uint32_t m = code - 1u;
    return (m & 1u) ? (int32_t)((m + 1u) >> 1) : -(int32_t)(m >> 1);
}

// minus the width of a code with z leading zeros, -(2 z + 1), as one v_mad_i32_i24.  Its low 5 bits are
// 32 - the width: the shift amount of v_lshrrev / v_alignbit (which read only those bits) that takes the
// code off the top of a 32-bit window, and the sum of a step's values is minus the bits it took.
__device__ __forceinline__ int32_t eg_negwidth(uint32_t z) {
    int32_t r;
    asm("v_mad_i32_i24 %0, %1, -2, -1" : "=v"(r) : "v"(z));
    return r;
}

// The code at window bit q (any valid width, up to 63 bits): the rare long code of parse_step
__device__ __forceinline__ uint32_t win_code_at(const uint32_t* win, uint32_t& q) {
    const uint32_t k = q >> 5, sh = q & 31u;
    const uint64_t h = (((uint64_t)win[k] << 32) | win[k + 1]) << sh;
    const uint64_t x = sh ? (h | (win[k + 2] >> (32u - sh))) : h;
    const uint32_t w = 2u * (uint32_t)__builtin_clzll(x) + 1u;  // a validated stream: < 32 leading zeros
    q += w;
    return (uint32_t)(x >> (64u - w));
}

// One parse step of a validated stream in an LDS window: C codes from window bit p, read from the window
// itself.  Words k - 1 .. k + C - 1 (k = ceil(p / 32)) funnel-shifted by p mod 32 hold the 32 C bits at p,
// and C codes of <= 31 bits (|v| < 2^15: every code an encoder of 8-bit frames writes) take at most 31 C
// of them.  No buffer is carried between steps, so no refill test and no divergent refill branch: a step
// is one round of LDS reads, C funnel shifts, and per code a leading-zero count, a shift and the funnel
// shifts of the bits behind it.  win[-1] must be readable (the window starts one word into its region):
// it is read, and ignored, at p = 0.
// The position is carried negated, n = -p: the funnel shift (32 - p mod 32) mod 32 is n's low 5 bits
// (alignbit reads no others), k = -(n >> 5) (arithmetic shift), and n moves by the codes' negated widths
// (eg_negwidth), which are their shift amounts too -- the step's address is a shift and an add, its
// position update two three-operand adds (round 5: p's ceiling, shift and update were 9 VALU of ~34).
// CHECK: a code of 33+ bits may occur (the mark pass saw one: status[3]); the step's codes are then
// re-read at their positions when one of them is that long (wave-uniform test).  Otherwise no code is.
template <int C, bool CHECK>
__device__ __forceinline__ void parse_step(const uint32_t* win, int32_t& n, uint32_t (&code)[C]) {
    const uint32_t* w = (const uint32_t*)((const char*)win + __mul24(n >> 5, -4));
    const uint32_t s = (uint32_t)n;
    uint32_t x[C + 1], b[C];
    int32_t nw[C];
#pragma unroll
    for (int j = 0; j <= C; j++) x[j] = w[j - 1];
#pragma unroll
    for (int j = 0; j < C; j++) b[j] = __builtin_amdgcn_alignbit(x[j], x[j + 1], s);
    uint32_t mn = 0xFFFFFFFFu;
#pragma unroll
    for (int e = 0; e < C; e++) {
        nw[e] = eg_negwidth(__builtin_clz(b[0]));
        code[e] = b[0] >> ((uint32_t)nw[e] & 31u);  // the low 5 bits: 32 - width (v_lshrrev reads no others)
        if constexpr (CHECK) mn = min(mn, b[0]);
#pragma unroll
        for (int j = 0; j + 1 < C - e; j++) b[j] = __builtin_amdgcn_alignbit(b[j], b[j + 1], (uint32_t)nw[e]);
    }
    int32_t sum = 0;
#pragma unroll
    for (int e = 0; e < C; e++) sum += nw[e];
    if (CHECK && __builtin_expect(__ballot(mn < 0x10000u) != 0ull, 0)) {  // a code of 33+ bits
        uint32_t p = (uint32_t)-n;
#pragma unroll
        for (int e = 0; e < C; e++) code[e] = win_code_at(win, p);
        n = -(int32_t)p;
    } else {
        n += sum;
    }
}

// A consumer lane's N codes from window bit p: four per step (the window carries 5 words of slack past
// the last mark: a step reads up to word ceil(p / 32) + 3)
#ifndef DCT3D_PARSE_C
#define DCT3D_PARSE_C 4
#endif
template <int N, bool CHECK>
__device__ __forceinline__ void parse_win(const uint32_t* win, uint32_t p, uint32_t (&cd)[N]) {
    constexpr int C = DCT3D_PARSE_C;
    static_assert(N % C == 0, "whole steps");
    int32_t n = -(int32_t)p;
#pragma unroll
    for (int i = 0; i < N; i += C) {
        uint32_t c[C];
        parse_step<C, CHECK>(win, n, c);
#pragma unroll
        for (int e = 0; e < C; e++) cd[i + e] = c[e];
    }
}

// A consumer lane's N codes (not values: eg_value_fast, or the decode's dequantisation, converts) from
// stream bit `my` (a mark: the stream is validated by the mark pass).  long_codes (status[3], grid-uniform):
// the stream holds a code of 33+ bits.  fits (wave-uniform): the wave's bit range is staged in its LDS
// window (words [w0, w0 + nwin), win[-1] readable: parse_step); else the parse reads the stream in global
// memory -- a wave whose 2,048 values average more than the window holds (|q| >= 2^13 nearly everywhere:
// never written by an encoder of 8-bit frames, but a valid stream).  That path's codes pass through the
// (then unused) window region, lane-private rows of N words (64 N words: every caller's region holds
// them), so that cd is written at constant indices only (a runtime index into cd would make a caller's
// loop carry all of cd: decode_eg_kernel).
// p: the lane's first bit relative to bit 32 w0 (the window's first).
template <int N>
__device__ __forceinline__ void parse_codes(const EgDecParams& P, uint32_t* win, uint32_t nwin, uint64_t w0,
                                            bool fits, bool long_codes, uint32_t p, uint32_t (&cd)[N]) {
    if (fits) {
        if (long_codes) parse_win<N, true>(win, p, cd);
        else parse_win<N, false>(win, p, cd);
    } else {
        const uint64_t my = w0 * 32 + p;
        uint32_t* row = (win - 1) + (threadIdx.x & 63) * N;  // from the region's first word
        BitReader<GlobalBits> r{GlobalBits{P.words, P.n_words}, 0, 0, 0, 0, 0};
        r.seek(my);
        for (int i = 0; i < N; i++) {
            uint32_t code = 1u;
            (void)r.get(code);
            row[i] = code;
        }
#pragma unroll
        for (int i = 0; i < N; i++) cd[i] = row[i];
    }
}

}  // namespace dct3d
