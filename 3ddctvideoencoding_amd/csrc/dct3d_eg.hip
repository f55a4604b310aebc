// dct3d_eg.hip -- the signed order-0 Exp-Golomb stage on the device.
//
// Replaces applyExpGolombCoding (encoder.c:60-71) over expGolomb_writeValue (ExpGolomb.c:32-64) and
// the Java writer (ExpGolombWriter.java:19-49, Encoder.java:91-111): every cube's quantised values in
// diagonal-slice order (cubeUtils_diagonalSlices, CubeUtils.c:5-46), each mapped v <= 0 -> -2v,
// v > 0 -> 2v - 1, plus one, written as (n - 1) zero bits followed by the n-bit value, MSB first, all
// cubes back to back in one bitstream that continues the caller's partial byte.
//
// Placement of variable-length codes without a serial cursor:
//   eg_len_kernel     one wave per cube: bits of the cube (sum of 2n - 1)
//   scan kernels      64-bit exclusive prefix sum over cubes (reduce / top / apply), plus the total
//   eg_write_kernel   waves walk the cubes (next cube prefetched): lane-level exclusive scan of code
//                     lengths, codes OR-ed into a wave-private LDS image aligned to the cube's first
//                     output word, stored as stream-order words (byte-swapped); interior words are
//                     plain stores, the first and last word go to head / tail
//   eg_stitch_kernel  merges the words shared by neighbouring cubes (and the carried partial byte)
#include <hip/hip_runtime.h>

#include <cstdint>

#include "dct3d_eg_bits.h"
#include "dct3d_kernels.h"

namespace dct3d {
namespace {

constexpr int kEgBlock = 256;
constexpr int kEgWaves = kEgBlock / 64;
constexpr int kScanChunk = 4096;              // cubes per scan block (16 per thread)

// code of one value: returns the n-bit value (v <= 0 -> -2v, else 2v - 1, plus one); *width = 2n - 1.
// Valid for |v| < 2^30 (quantised 8-bit content stays below 2^13); flags anything larger.
__device__ __forceinline__ uint32_t eg_code(int32_t v, int& width, bool& bad) {
    bad |= (v >= (1 << 30)) | (v <= -(1 << 30));
    const uint32_t m = v <= 0 ? (uint32_t)(-2 * v) : (uint32_t)(2 * v - 1);
    const uint32_t code = m + 1u;
    const int n = 32 - __clz((int)code);
    width = 2 * n - 1;
    return code;
}

__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
    return x;
}

template <int D>
__global__ __launch_bounds__(kEgBlock) void eg_len_kernel(EgParams P) {
    constexpr int CS = 64 * D, PER = CS / 64;
    const int lane = threadIdx.x & 63;
    const uint64_t g = (uint64_t)blockIdx.x * kEgWaves + (threadIdx.x >> 6);
    if (g >= P.n_cubes) return;
    const int32_t* q = P.q + g * CS + lane * PER;
    uint32_t bits = 0;
    bool bad = false;
#pragma unroll
    for (int i = 0; i < PER; i += 4) {
        const int4 v = *(const int4*)(q + i);
        const int32_t vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int e = 0; e < 4; e++) {
            int w;
            (void)eg_code(vv[e], w, bad);
            bits += (uint32_t)w;
        }
    }
    if (__ballot(bad) != 0ull && lane == 0) atomicOr((unsigned int*)&P.status[1], 2u);
    bits = wave_sum_u32(bits);
    if (lane == 0) P.bits[g] = bits;
}

// block b: sum of bits over its chunk of kScanChunk cubes (coalesced: thread t takes t, t + 256, ...;
// strided by thread before: 15 -> 6 us per c8 step)
__global__ __launch_bounds__(kEgBlock) void eg_scan_reduce_kernel(EgParams P) {
    __shared__ uint64_t part[kEgWaves];
    const uint64_t base = (uint64_t)blockIdx.x * kScanChunk + threadIdx.x;
    uint32_t v[kScanChunk / kEgBlock];
#pragma unroll
    for (int i = 0; i < kScanChunk / kEgBlock; i++)  // all loads in flight first
        v[i] = base + i * kEgBlock < P.n_cubes ? P.bits[base + i * kEgBlock] : 0u;
    uint64_t s = 0;
#pragma unroll
    for (int i = 0; i < kScanChunk / kEgBlock; i++) s += v[i];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t t = 0;
        for (int w = 0; w < kEgWaves; w++) t += part[w];
        P.bsum[blockIdx.x] = t;
    }
}

// The stream decode's reduce (round 6: replaces the apply kernel and its 8-byte offset per chunk): block b
// sums the counts of chunks 4096 b .. 4096 b + 4095 into bsum[b] (then scanned by eg_scan_top_kernel) and
// each 256 of them into part[16 b + i] (thread t holds the 16 consecutive counts 16 t ..: a part is 16
// lanes).  The mark pass adds the parts before its block and scans its own 256 counts.
__global__ __launch_bounds__(kEgBlock) void eg_dscan_reduce_kernel(EgDecParams P) {
    static_assert(kScanChunk == 16 * kEgBlock && kEgBlock == 256, "16 counts per thread, 16 parts per block");
    __shared__ uint32_t wsum[kEgWaves];
    const uint64_t base = (uint64_t)blockIdx.x * kScanChunk + threadIdx.x * 16u;
    uint32_t s = 0;
    if (base + 16 <= P.n_chunks) {
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const uint4 t = *(const uint4*)(P.count + base + 4 * q);
            s += t.x + t.y + t.z + t.w;
        }
    } else {
        for (uint32_t i = 0; i < 16; i++) s += base + i < P.n_chunks ? P.count[base + i] : 0u;
    }
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) s += __shfl_xor(s, o, 64);  // the part: 16 lanes
    if ((lane & 15) == 0) P.part[(uint64_t)blockIdx.x * 16 + wave * 4 + lane / 16] = s;
    s += __shfl_xor(s, 16, 64);
    s += __shfl_xor(s, 32, 64);
    if (lane == 0) wsum[wave] = s;
    __syncthreads();
    if (threadIdx.x == 0) P.bsum[blockIdx.x] = (uint64_t)wsum[0] + wsum[1] + wsum[2] + wsum[3];
}

// one block: exclusive scan of the chunk sums (offset by the carried bits), total, capacity check.  Thread t
// owns the consecutive sums t K .. t K + K - 1 (K = ceil(n / 1024)): their serial sum, one block scan of the
// 1,024 sums (in the wave by shuffles, the 16 waves' totals through LDS), then its prefixes written back.
// (Round 6; a Hillis-Steele pass per 1,024 sums before: 20 barriers each, 5 / 9 us per c8 step.)
__global__ __launch_bounds__(1024) void eg_scan_top_kernel(EgParams P, uint32_t n_chunks) {
    __shared__ uint64_t wsum[16];
    const uint32_t K = (n_chunks + 1023) / 1024;
    const uint32_t i0 = threadIdx.x * K;
    uint64_t s = 0;
    for (uint32_t i = i0; i < i0 + K && i < n_chunks; i++) s += P.bsum[i];
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint64_t incl = s;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t t = __shfl_up(incl, o, 64);
        if (lane >= (uint32_t)o) incl += t;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    uint64_t run = (uint64_t)P.carry_bits + incl - s, total = P.carry_bits;
    for (uint32_t w = 0; w < 16; w++) {
        run += w < wave ? wsum[w] : 0u;
        total += wsum[w];
    }
    for (uint32_t i = i0; i < i0 + K && i < n_chunks; i++) {
        const uint64_t v = P.bsum[i];
        P.bsum[i] = run;
        run += v;
    }
    if (threadIdx.x == 0) {
        P.status[0] = total;  // total bits including the carried ones
        if ((total + 31) / 32 > P.out_cap_words) atomicOr((unsigned int*)&P.status[1], 1u);
    }
}

// block b: per-cube exclusive offsets inside the chunk, plus the chunk's offset.  Thread t owns the 16
// consecutive entries 16 t .. 16 t + 15 (four 16-byte loads, eight 16-byte stores of a whole 128-byte
// line of offsets); the threads' sums are scanned in the wave by shuffles and across the block's 4 waves
// through LDS (one barrier; a Hillis-Steele scan over the 256 threads took 16 barriers: 39 -> 18 us per
// c8 step).
__global__ __launch_bounds__(kEgBlock) void eg_scan_apply_kernel(EgParams P) {
    constexpr int PER = kScanChunk / kEgBlock;
    static_assert(PER == 16, "four 16-byte loads per thread");
    __shared__ uint64_t wsum[kEgWaves];
    const uint64_t base = (uint64_t)blockIdx.x * kScanChunk + threadIdx.x * PER;
    const uint64_t boff = P.bsum[blockIdx.x];
    uint32_t v[PER];
    if (base + PER <= P.n_cubes) {  // (bits holds n_cubes entries; off as many)
#pragma unroll
        for (int q = 0; q < PER / 4; q++) {
            const uint4 t = *(const uint4*)(P.bits + base + 4 * q);
            v[4 * q] = t.x; v[4 * q + 1] = t.y; v[4 * q + 2] = t.z; v[4 * q + 3] = t.w;
        }
    } else {
#pragma unroll
        for (int i = 0; i < PER; i++) v[i] = base + i < P.n_cubes ? P.bits[base + i] : 0u;
    }
    uint64_t s = 0;
#pragma unroll
    for (int i = 0; i < PER; i++) s += v[i];
    // inclusive scan of the threads' sums within the wave
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint64_t incl = s;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t t = __shfl_up(incl, o, 64);
        if (lane >= o) incl += t;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    uint64_t run = boff + incl - s;
    for (int w = 0; w < wave; w++) run += wsum[w];
    if (base + PER <= P.n_cubes) {
#pragma unroll
        for (int i = 0; i < PER; i += 2) {
            const uint64_t a = run;
            run += v[i];
            const uint64_t b = run;
            run += v[i + 1];
            *(ulonglong2*)(P.off + base + i) = make_ulonglong2(a, b);
        }
    } else {
#pragma unroll
        for (int i = 0; i < PER; i++) {
            if (base + i < P.n_cubes) P.off[base + i] = run;
            run += v[i];
        }
    }
}

// OR of one code into a word image: the n-bit value ends at stream bit e (exclusive, relative to
// word 0 of the image); at most two words
template <class OrFn>
__device__ __forceinline__ void put_code(uint32_t code, int width, uint32_t e, OrFn&& or_word) {
    const uint32_t n = ((uint32_t)width + 1) >> 1;
    const uint32_t kl = (e - 1) >> 5;
    const uint32_t r = e - 32 * kl;  // 1..32 bits of the value in word kl
    or_word(kl, code << (32 - r));
    if (n > r) or_word(kl - 1, code >> r);
}

// Each wave walks cubes g = wave_id, wave_id + n_waves, ... with the next cube's values and offset
// prefetched while the current one is packed.  A cube's words are assembled in a 256-word LDS image
// (8,160 bits: 16x what quantised content needs; larger cubes, up to 512 x 63 bits, take several
// windows).  Interior words are plain stores; the first and the last word, which the cube may share
// with its neighbours, go to head[g] / tail[g] for eg_stitch_kernel -- no global atomics, and every
// output word is written exactly once (no zero fill).  A cube has >= 512 bits (>= 16 words), so a
// word is shared by at most two cubes.
constexpr int kImgWords = 256;
template <int D>
__global__ __launch_bounds__(kEgBlock) void eg_write_kernel(EgParams P) {
    constexpr int CS = 64 * D, PER = CS / 64, V4 = PER / 4;
    __shared__ int32_t sq[kEgWaves][CS];
    __shared__ uint32_t img[kEgWaves][kImgWords];
    if (P.status[1] != 0) return;  // capacity or range failure: nothing is written
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t n_waves = (uint64_t)gridDim.x * kEgWaves;
    uint64_t g = (uint64_t)blockIdx.x * kEgWaves + wave;
    if (g >= P.n_cubes) return;
    uint16_t dg[PER];
#pragma unroll
    for (int i = 0; i < PER; i++) dg[i] = P.diag[lane * PER + i];
    int4 nxt[V4];
#pragma unroll
    for (int i = 0; i < V4; i++) nxt[i] = *(const int4*)(P.q + g * CS + i * 256 + lane * 4);
    uint64_t nxt_off = P.off[g];
    for (; g < P.n_cubes; g += n_waves) {
#pragma unroll
        for (int i = 0; i < V4; i++) *(int4*)&sq[wave][i * 256 + lane * 4] = nxt[i];
        const uint64_t start = nxt_off;
        const uint64_t gn = g + n_waves;
        if (gn < P.n_cubes) {  // next cube's values and offset in flight while this one is packed
#pragma unroll
            for (int i = 0; i < V4; i++) nxt[i] = *(const int4*)(P.q + gn * CS + i * 256 + lane * 4);
            nxt_off = P.off[gn];
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        uint32_t code[PER];
        int width[PER];
        bool bad = false;
        uint32_t lbits = 0;
#pragma unroll
        for (int i = 0; i < PER; i++) {
            code[i] = eg_code(sq[wave][dg[i]], width[i], bad);
            lbits += (uint32_t)width[i];
        }
        uint32_t incl = lbits;  // exclusive scan of the lanes' bit counts (stream order = lane order)
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t t = __shfl_up(incl, o, 64);
            if (lane >= o) incl += t;
        }
        const uint32_t total = __shfl(incl, 63, 64);
        const uint32_t s0 = (uint32_t)(start & 31);
        const uint64_t w0 = start >> 5;
        const uint32_t nwords = (s0 + total + 31) >> 5;
        const uint32_t pos0 = s0 + incl - lbits;  // stream bit of this lane's first code, relative to w0
        for (uint32_t win = 0; win < nwords; win += kImgWords) {
            const uint32_t nw = min(nwords - win, (uint32_t)kImgWords);
            for (uint32_t w = lane; w < nw; w += 64) img[wave][w] = 0u;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            uint32_t pos = pos0;
#pragma unroll
            for (int i = 0; i < PER; i++) {
                pos += (uint32_t)width[i];
                put_code(code[i], width[i], pos, [&](uint32_t k, uint32_t v) {
                    if (k - win < nw) atomicOr(&img[wave][k - win], v);  // unsigned: k >= win
                });
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            for (uint32_t w = lane; w < nw; w += 64) {
                const uint32_t gw = win + w;
                const uint32_t v = __builtin_bswap32(img[wave][w]);  // stream order -> memory byte order
                if (gw == 0) P.head[g] = v;
                else if (gw == nwords - 1) P.tail[g] = v;
                else P.out[w0 + gw] = v;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // img / sq reuse
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
    }
}

// thread per cube: the first word of cube g = its head | the previous cube's tail when they share the
// word (| the carried partial byte for g = 0); the last word (tail) unless the next cube shares it
__global__ __launch_bounds__(kEgBlock) void eg_stitch_kernel(EgParams P) {
    if (blockIdx.x == 0 && threadIdx.x < 2) {
        if (P.status_host) P.status_host[threadIdx.x] = P.status[threadIdx.x];
        if (P.status_clear) P.status_clear[threadIdx.x] = 0u;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0 && P.status_host && P.seq)  // the verdict as one tag word
        __hip_atomic_store(P.status_host + 7, hand_off_tag(P.seq, P.status[0], (uint32_t)(P.status[1] & 3u)),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (P.status[1] != 0) return;
    const uint64_t g = (uint64_t)blockIdx.x * kEgBlock + threadIdx.x;
    if (g >= P.n_cubes) return;
    const uint64_t start = P.off[g], end = start + P.bits[g];
    if (end == start) return;  // never for a coded cube or segment (>= 256 bits); no word to place
    const uint64_t w0 = start >> 5, wl = (end - 1) >> 5;
    uint32_t first = P.head[g];
    if (g == 0) first |= P.carry_byte & (0xFF00u >> P.carry_bits);  // stream byte 0 = memory byte 0
    else if (((start - 1) >> 5) == w0) first |= P.tail[g - 1];
    P.out[w0] = first;
    if (g + 1 == P.n_cubes || (end >> 5) != wl) P.out[wl] = P.tail[g];
}

// Fused path, K3: kCompactSPW consecutive segments (8 cubes each, coded by encode_eg_kernel) per wave.
// The slot holds a segment's stream, its first bit at bit 31 of word 0 (K1 places every lane's codes at
// the lane's bit offset in the segment), so the segment's words only move to its stream offset off[s]:
// output word i = slot words i - 1 and i funnel-shifted by off[s] mod 32, byte-swapped, lane j handling
// words j, j + 64, ... (consecutive words per store instruction).  kCompactPF rows of 64 words of every
// segment of the wave per load round trip (a segment of 1080p ramp content: ~180 words, uniform noise
// ~420).  The first and the last word of a segment,
// which it may share with its neighbours, go to head / tail for eg_stitch_kernel, like a cube of
// eg_write_kernel.  (Round 4 before: lane-local words in slot columns and a lane bit-count array, the
// lanes concatenated here through shuffles and an LDS image: 275 us per c7 step, 0.42 GB of slot reads;
// one segment per wave: 201 us, two dependent round trips per 180 words.)
constexpr int kCompactPF = 4;   // rows of 64 words per segment per load round trip
constexpr int kCompactSPW = 4;  // segments per wave
__global__ __launch_bounds__(kEgBlock) void eg_compact_kernel(EgParams P, const uint32_t* __restrict__ slot,
                                                              uint32_t seg_cap) {
    if (P.status[1] != 0) return;  // capacity failure: nothing is written
    const int lane = threadIdx.x & 63;
    // wave-uniform (scalar) segment index, offsets and sizes; 32-bit lane offsets
    const uint32_t s0 = (uint32_t)__builtin_amdgcn_readfirstlane(
        (int)((blockIdx.x * kEgWaves + (threadIdx.x >> 6)) * kCompactSPW));
    if (s0 >= P.n_cubes) return;
    uint64_t base[kCompactSPW];
    uint32_t nsrc[kCompactSPW], ndst[kCompactSPW];
#pragma unroll
    for (int t = 0; t < kCompactSPW; t++) {
        const bool live = s0 + t < P.n_cubes;
        base[t] = live ? P.off[s0 + t] : 0;
        const uint32_t tot = live ? P.bits[s0 + t] : 0u;  // >= 256 for a live segment (a whole cube)
        nsrc[t] = (tot + 31) >> 5;
        ndst[t] = tot ? (uint32_t)(((base[t] + tot - 1) >> 5) - (base[t] >> 5) + 1) : 0u;
    }
    auto load_rows = [&](int t, uint32_t i0, uint32_t (&cur)[kCompactPF], uint32_t (&prv)[kCompactPF]) {
        const uint32_t* seg = slot + (uint64_t)(s0 + t) * seg_cap;
#pragma unroll
        for (int r = 0; r < kCompactPF; r++) {  // word i - 1: an L1 hit
            const uint32_t i = i0 + r * 64 + lane;
            cur[r] = i < nsrc[t] ? seg[i] : 0u;
            prv[r] = i - 1u < nsrc[t] ? seg[i - 1u] : 0u;  // i = 0: none
        }
    };
    auto store_rows = [&](int t, uint32_t i0, const uint32_t (&cur)[kCompactPF], const uint32_t (&prv)[kCompactPF]) {
        const uint32_t r = (uint32_t)(base[t] & 31);
        uint32_t* const outs = P.out + (base[t] >> 5);
#pragma unroll
        for (int k = 0; k < kCompactPF; k++) {
            const uint32_t i = i0 + k * 64 + lane;
            if (i < ndst[t]) {
                const uint32_t v = __builtin_bswap32(__builtin_amdgcn_alignbit(prv[k], cur[k], r));
                if (i == 0) P.head[s0 + t] = v;
                else if (i == ndst[t] - 1) P.tail[s0 + t] = v;
                else outs[i] = v;
            }
        }
    };
    uint32_t nmax = 0;
#pragma unroll
    for (int t = 0; t < kCompactSPW; t++) nmax = max(nmax, ndst[t]);
    for (uint32_t i0 = 0; i0 < nmax; i0 += kCompactPF * 64) {  // all segments' rows in flight together
        uint32_t cur[kCompactSPW][kCompactPF], prv[kCompactSPW][kCompactPF];
#pragma unroll
        for (int t = 0; t < kCompactSPW; t++) load_rows(t, i0, cur[t], prv[t]);
#pragma unroll
        for (int t = 0; t < kCompactSPW; t++) store_rows(t, i0, cur[t], prv[t]);
    }
}

// =================================================================================================
// Decode: the inverse of the stream above (expGolomb_readValue, ExpGolomb.c:66-110 /
// ExpGolombReader.java:19-63; Decoder.java:78-96 places value i of a cube at diagonal position i).
// Self-synchronising parallel decode: the stream is cut into kChunkBits chunks, one thread each.
//   sync pass k   thread t parses codewords from its start (k = 0: the chunk's first bit; later: the
//                 previous pass's exit of chunk t - 1) until it passes the chunk's end; exit = the
//                 first codeword boundary at or past the end.  Repeated until no exit changes: chunk 0
//                 starts at the true first bit, so by induction every start is then a true boundary.
//                 Exp-Golomb parses resynchronise within a few codewords, so two passes are typical.
//   scan          value index of each chunk's first codeword
//   mark pass     each chunk parsed once more from its (true) start: the bit position of every 32nd
//                 value goes to mark[idx / 32]; the end bit of value n_values - 1 is recorded
//   emit          one wave per 2,048 values (4 cubes of 8x8x8 / 8 of 8x8x4): lane l parses the 32
//                 values from mark[l]; the wave scatters them to their diagonal positions in LDS and
//                 writes the cubes with 1 KiB coalesced stores
// The parses read the stream from LDS: the block (sync, mark) or the wave (emit) first stages its
// contiguous bit range with coalesced loads.  (A parse reading global memory waits a full memory
// round trip at nearly every code: some lane of the wave refills on ~94 % of the codes, and the
// wave-wide vmcnt cannot wait for one lane's word only.  A per-value scatter of the values to their
// cubes -- 2.1 G single-dword stores per 128 stacks -- took 47 ms.)
// A parse that meets 32 zero bits (no valid code has more than 30 leading zeros) ends "invalid":
// in a true parse inside the wanted values that means a corrupt stream.
constexpr uint64_t kChunkBits = kEgChunkBits;
constexpr uint64_t kNoExit = ~0ull;
static_assert(kChunkBits == 512 && kEgBlock == 256, "16-word chunks");
constexpr uint32_t kMarkVals = 32;          // values per emit lane / per mark
constexpr uint32_t kEmitWinWords = 2048;    // per wave: window (<= 2,048 values x 27 bits) / 8 KiB staging

// ---------------------------------------------------------------------------------------------------------
// The block's window as chunk columns (round 6).  A thread parses one 512-bit chunk; its reads wander over
// its chunk, so in a linear window (rounds 1-5) the 32 lanes of a read's lane group sat 16 words apart on
// 2 of the 32 banks of ds_read_b32 (MI355X_MICROARCH.md §LDS) until their offsets drifted apart: 6-8
// conflict cycles per LDS instruction (profiles/r05/sq_c8_summary*.csv).  Column c of the window holds
// chunk first + c shifted to start at bit 31 of its word 0, plus the first two words of the next chunk
// (kColW words: every read of the lean and bounded steps), word j of column c at LDS word
// (c / 32) * 32 kColW + 32 j + c % 32: a lane's reads all fall on bank c % 32, so a lane group's reads
// never conflict, and word j of a column is one stride of 128 bytes from word j - 1, so the column read is
// as cheap to address as a linear one (col_bits64).  Positions are chunk-relative 32-bit bits (0 = the
// chunk's nominal first bit).  The rare checked steps that read past the column (a code of >= 33 bits
// crossing the chunk end, the data's end) read the stream in global memory (ColReader).
constexpr uint32_t kColW = 18;
constexpr uint32_t kColBytes = kEgBlock * kColW * 4;
static_assert(kEgBlock % 32 == 0, "whole lane groups of columns");

// LDS of the three front kernels, carved by hand so that the table sits right before the window (a
// column's word -1, read and ignored by col_bits64 at p = 0, is then table bytes): table | window | ...
constexpr uint32_t kLutBytes = 1u << 12;

// The window of chunks first + c, c < kEgBlock (first may be -1: block 0 of the resolving pass), then the
// caller's barrier.  Thread c loads its chunk's words (four 16-byte loads + three, all in flight at once),
// funnel-shifts them by the stream's bit offset and writes them down its column.  Words past the stream
// (or before it: chunk -1) are zero.  PAD: words in front of each column (the mark pass's first mark
// slots); a group of 32 columns then spans 32 (kColW + PAD) words.
template <uint32_t PAD = 0>
__device__ __forceinline__ void stage_columns(const EgDecParams& P, uint32_t* win, int64_t first) {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4), aligned(4)));
    const int64_t b0 = (int64_t)P.start_bit + (first + (int64_t)threadIdx.x) * (int64_t)kChunkBits;
    const int64_t w = b0 >> 5;  // arithmetic: floor
    const uint32_t o = (uint32_t)b0 & 31u;  // the same for every chunk of the stream (block-uniform)
    uint32_t g[kColW + 1];
    if (w >= 0 && (uint64_t)w + kColW + 1 <= P.n_words) {
        const uint32_t* src = P.words + w;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const u32x4 x = *(const u32x4*)(src + 4 * q);
            g[4 * q] = x[0]; g[4 * q + 1] = x[1]; g[4 * q + 2] = x[2]; g[4 * q + 3] = x[3];
        }
#pragma unroll
        for (uint32_t j = 16; j <= kColW; j++) g[j] = src[j];
    } else {
#pragma unroll
        for (uint32_t j = 0; j <= kColW; j++) {
            const int64_t k = w + (int64_t)j;
            g[j] = k >= 0 && (uint64_t)k < P.n_words ? P.words[k] : 0u;
        }
    }
#pragma unroll
    for (uint32_t j = 0; j <= kColW; j++) g[j] = __builtin_bswap32(g[j]);
    uint32_t* col = win + (threadIdx.x >> 5) * (32 * (kColW + PAD)) + 32 * PAD + (threadIdx.x & 31);
    if (o) {
#pragma unroll
        for (uint32_t j = 0; j < kColW; j++) col[32 * j] = __builtin_amdgcn_alignbit(g[j], g[j + 1], 32u - o);
    } else {
#pragma unroll
        for (uint32_t j = 0; j < kColW; j++) col[32 * j] = g[j];
    }
}
template <uint32_t PAD = 0, typename W>
__device__ __forceinline__ W* column(W* win) {
    return win + (threadIdx.x >> 5) * (32 * (kColW + PAD)) + 32 * PAD + (threadIdx.x & 31);
}

// chunk-relative form of an absolute bit position (clamped to [0, 2^32 - 1])
__device__ __forceinline__ uint32_t rel_bit(uint64_t p, int64_t b0) {
    if (b0 >= 0 && p <= (uint64_t)b0) return 0u;
    const uint64_t d = p - (uint64_t)b0;
    return d >= 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)d;
}

// 32 stream bits at absolute bit a (MSB first; zero past the stream): the checked steps' rare global reads
__device__ __forceinline__ uint32_t stream_bits32(const EgDecParams& P, uint64_t a) {
    const uint64_t k = a >> 5;
    const uint32_t o = (uint32_t)a & 31u;
    const uint32_t x = stream_word(P, k), y = stream_word(P, k + 1);
    return o ? __builtin_amdgcn_alignbit(x, y, 32u - o) : x;
}

// The buffered one-code-at-a-time reader of the checked steps (as BitReader, dct3d_eg_bits.h) over a column:
// word i < kColW from LDS, beyond from the stream in global memory.
struct ColReader {
    const uint32_t* col;
    const EgDecParams* P;
    uint64_t b0;     // absolute bit of the column's bit 0 (a live chunk: >= 0)
    uint32_t next;   // index of the word held in `pre`
    uint64_t buf;    // left-aligned bits [pos, pos + avail)
    int avail;
    uint32_t pos;
    uint32_t pre;
    __device__ __forceinline__ uint32_t word(uint32_t i) const {
        if (i < kColW) return col[32 * i];
        return stream_bits32(*P, b0 + 32ull * i);
    }
    __device__ __forceinline__ void seek(uint32_t p) {
        pos = p;
        const uint32_t k = p >> 5;
        const int sh = (int)(p & 31);
        buf = (((uint64_t)word(k) << 32) | word(k + 1)) << sh;
        avail = 64 - sh;
        next = k + 2;
        pre = word(next);
    }
    __device__ __forceinline__ void refill() {
        if (avail <= 32) {
            buf |= (uint64_t)pre << (32 - avail);
            avail += 32;
            pre = word(++next);
        }
    }
    // a run of 1-bit codes (value 0), at most maxn, stopping where the buffered bits end
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
    // one codeword (any width up to 63 bits): false when 32 zero bits come first (invalid)
    __device__ __forceinline__ bool get(uint32_t& code) {
        refill();
        const uint32_t hi32 = (uint32_t)(buf >> 32);
        if (hi32 == 0u) return false;
        const int width = 2 * __builtin_clz(hi32) + 1;
        if (width <= avail) {
            code = (uint32_t)(buf >> (64 - width));
            buf <<= width;
            avail -= width;
            pos += (uint32_t)width;
        } else {  // a long code straddling the buffer: read it at its position
            const uint32_t k = pos >> 5;
            const int sh = (int)(pos & 31);
            const uint64_t hi = (((uint64_t)word(k) << 32) | word(k + 1)) << sh;
            const uint64_t x = sh ? (hi | ((uint64_t)word(k + 2) >> (32 - sh))) : hi;
            code = (uint32_t)(x >> (64 - width));
            seek(pos + (uint32_t)width);
        }
        return true;
    }
};

// A parse from a wrong start meets the true parse (a boundary of both) within 90 bits on every one of
// 10.7 k chunks of the 1080p content (within 64 bits on 99.57 %, at the chunk start on half of them).
constexpr uint32_t kMeetBits = 128;

// One checked parse step (a run of 1-bit codes, or one longer code): false once the parse has ended (at
// `stop`, or invalid).
__device__ __forceinline__ bool sync_step(ColReader& r, uint32_t stop, uint32_t limit, uint32_t& n, bool& invalid) {
    uint32_t code;
    const uint32_t k = r.ones(min(stop - r.pos, 64u));
    n += k;
    if (r.pos >= stop) return false;
    if (!r.at_long_code()) return true;  // the buffered bits ran out inside the run: refill
    if (!r.get(code) || r.pos > limit) {  // 32 zero bits, or a code running past the data
        invalid = true;
        return false;
    }
    n++;
    return true;
}

// The parse passes' chunk interiors: branchless steps read from the column at their position (round 6).
// Round 4 made the interior steps branchless (sync 625 -> 558 us, mark 896 -> 798 us per c8 step: every
// branch was exec-mask bookkeeping on the scalar unit that a wave ran whenever any lane took it); rounds 4-5
// carried a 64-bit buffer with its fill count and a one-word prefetch between steps, so every step paid a
// select-based refill (~10 VALU of 33 in the sync pass's table step).  Now a step carries only its position
// p and reads the 64 bits at p from its column -- words k - 1 .. k + 1, k = ceil(p / 32), two funnel
// shifts by (32 - p mod 32) mod 32 (the consumer's parse_step, dct3d_eg_bits.h): no refill, no fill count,
// no carried words; its LDS read sits on the step's dependent chain, conflict-free in the column layout.
__device__ __forceinline__ void col_bits64(const uint32_t* col, uint32_t p, uint32_t& hi, uint32_t& lo) {
    const int32_t n = -(int32_t)p;
    const uint32_t* w = (const uint32_t*)((const char*)col + __mul24(n >> 5, -128));
    const uint32_t x0 = w[-32], x1 = w[0], x2 = w[32];
    hi = __builtin_amdgcn_alignbit(x0, x1, (uint32_t)n);  // alignbit reads the shift's low 5 bits only
    lo = __builtin_amdgcn_alignbit(x1, x2, (uint32_t)n);
}
// leading zeros of x, 0xFFFFFFFF for x = 0 (the hardware's v_ffbh_u32; clz(0) is undefined in C++, and a
// zero top word means an invalid code here: >= 16 as an unsigned count)
__device__ __forceinline__ uint32_t ffbh_u32(uint32_t x) {
    uint32_t r;
    asm("v_ffbh_u32 %0, %1" : "=v"(r) : "v"(x));
    return r;
}

// The interior loops run while the parse is a margin short of every bound: a step takes at most 31 + 31
// bits (a run of <= 31 one-bit codes, then the table's <= 12 bits or one code of <= 31), so only those
// bits must stay short of the bound.  Interior steps (p < 512 - 64) read words <= 15, the bounded steps
// (p < 512) words <= 17: the column.  (Round 5: 128, the old window-read bound, before: sync 346 -> 311
// us, mark 464 -> 442 us per c8 step.)
constexpr uint32_t kLeanMargin = 64;
static_assert(31 + 31 < kLeanMargin && (kChunkBits + 31) / 32 + 1 < kColW, "steps stay in the column");

// Table step: a run of 1-bit codes (clz of the complement, at most 31), then every code complete in the
// next kEgLutBits bits at once from a 4 KiB LDS table of (codes, bits) per bit pattern; none complete (a
// code of more than kEgLutBits bits): one code by its leading zeros.  20 VALU (round 5's buffered form:
// 33).  The sync pass needs only the count and the exit, so the codes' boundaries are never formed.
// Table width 12 bits: a 13- or 14-bit sync table cost more blocks per CU than it saved, a 10- or 11-bit
// mark table took more steps (profiles/r05/sync_table_bits, mark_table_bits).
constexpr int kEgLutBits = 12;
static_assert((1u << kEgLutBits) == kLutBytes, "the carved table");
template <int B>
struct EgLut {
    uint8_t e[1 << B];  // codes complete within the pattern (low 4 bits), the bits they take (high 4)
};
template <int B>
constexpr EgLut<B> make_eg_lut() {
    EgLut<B> t{};
    for (int v = 0; v < (1 << B); v++) {
        int p = 0, k = 0;
        for (;;) {
            int z = 0;
            while (p + z < B && !((v >> (B - 1 - p - z)) & 1)) z++;
            if (p + 2 * z + 1 > B) break;
            p += 2 * z + 1;
            k++;
        }
        t.e[v] = (uint8_t)(k | (p << 4));
    }
    return t;
}
template <int B>
__device__ constexpr EgLut<B> kEgLutT = make_eg_lut<B>();
// the block's copy of the table: 16-byte pieces, ordered by the staging's barrier
template <int B = kEgLutBits>
__device__ __forceinline__ void copy_lut(uint8_t* s_lut) {
    constexpr uint32_t kBytes = 1u << B;
    if constexpr (kBytes < 16 * kEgBlock) {  // 11 bits: 8 bytes per thread
        static_assert(kBytes == 8 * kEgBlock, "whole 8-byte pieces per thread");
        *(uint2*)(s_lut + 8 * threadIdx.x) = *(const uint2*)(kEgLutT<B>.e + 8 * threadIdx.x);
    } else {
        static_assert(kBytes % (16 * kEgBlock) == 0, "whole 16-byte pieces per thread");
#pragma unroll
        for (uint32_t r = 0; r < kBytes / (16 * kEgBlock); r++)
            *(uint4*)(s_lut + 16 * (threadIdx.x + r * kEgBlock)) = *(const uint4*)(kEgLutT<B>.e + 16 * (threadIdx.x + r * kEgBlock));
    }
}
static_assert(kEgLutBits <= 15, "counts and widths fit 4 bits");

// A step that meets a code of >= 33 bits (or 32 zero bits) ends the interior loop with that code counted
// and its (meaningless) width added to p; the loop's caller takes both back (pos_step_undo), so the step
// needs no selects for the case.
__device__ __forceinline__ uint32_t pos_step_lut(const uint32_t* col, const uint8_t* lut, uint32_t& p, bool& bad,
                                                 uint32_t& w_last) {
    uint32_t hi, lo;
    col_bits64(col, p, hi, lo);
    const uint32_t n1 = __builtin_clz(~hi | 1u);  // run of 1-bit codes, at most 31
    const uint32_t th = (uint32_t)(((((uint64_t)hi << 32) | lo) << n1) >> 32);
    const uint32_t e = lut[th >> (32 - kEgLutBits)];
    const uint32_t k = e & 15u;
    const uint32_t zz = ffbh_u32(th);
    const bool kz = k == 0u;                 // no code complete in the table's bits: one code by clz
    bad = kz & (zz >= 16u);                  // >= 33 bits or invalid: the checked loop reads it
    w_last = kz ? 2u * zz + 1u : e >> 4;
    p += n1 + w_last;
    return n1 + max(k, 1u);
}
__device__ __forceinline__ void pos_step_undo(bool bad, uint32_t w_last, uint32_t& p, uint32_t& n) {
    if (bad) {  // the code the last step met: back to its first bit, uncounted
        p -= w_last;
        n -= 1u;
    }
}

// The mark pass's table step: pos_step_lut that stops on the step's one possible mark.  d0: the values
// before the next mark.  All k table codes are taken unless the step's values would pass 32 (two marks) or
// the mark falls on the table's second .. k-th code, whose bit offsets the table does not give; then only
// the first code (its width by clz).  The mark is then always the run's d0-th value or the first code: bit
// p0 + d0 of the step.  (Round 5: the table in the mark pass, 430 -> 356 us per c8 step, profiles/r05/mark_lut.)
template <int B = kEgLutBits>
__device__ __forceinline__ uint32_t pos_step_lut_mark(const uint32_t* col, const uint8_t* lut, uint32_t& p, bool& bad,
                                                      uint32_t d0, uint32_t& w_last) {
    uint32_t hi, lo;
    col_bits64(col, p, hi, lo);
    const uint32_t n1 = __builtin_clz(~hi | 1u);
    const uint32_t th = (uint32_t)(((((uint64_t)hi << 32) | lo) << n1) >> 32);
    const uint32_t e = lut[th >> (32 - B)];
    const uint32_t k = e & 15u;
    const uint32_t zz = ffbh_u32(th);
    // (bitwise, not short-circuit: the compiler made branches of &&)
    const bool full = (k != 0u) & (n1 + k <= 32u) & (d0 - n1 - 1u >= k - 1u);
    bad = !full & (zz >= 16u);  // counted and taken back by the caller (pos_step_undo), as pos_step_lut
    const uint32_t wt = e >> 4, w1 = 2u * zz + 1u;
    w_last = full ? wt : w1;
    p += n1 + w_last;
    return n1 + (full ? k : 1u);
}

// Bounded table steps to the chunk end (round 6; rounds 4-5 took one run and one code per bounded step,
// ~9 steps over the last 64 bits of ramp content): the run is capped at the bits left before the stop, the
// table's codes are taken when they all end at or before it (no code boundary at or past the stop is
// skipped), else the one code after the run if it starts before the stop.  So the parse still ends
// exactly at the first code boundary at or past the stop.  bad: as pos_step_lut, but the code is left
// unconsumed (the checked loop reads it).
__device__ __forceinline__ uint32_t pos_step_lut_bounded(const uint32_t* col, const uint8_t* lut, uint32_t& p, bool& bad,
                                                         uint32_t stop) {
    const uint32_t room = stop - p;
    uint32_t hi, lo;
    col_bits64(col, p, hi, lo);
    const uint32_t n1 = __builtin_clz(~hi | (0x80000000u >> min(room, 31u)));
    const uint32_t th = (uint32_t)(((((uint64_t)hi << 32) | lo) << n1) >> 32);
    const uint32_t e = lut[th >> (32 - kEgLutBits)];
    const uint32_t k = e & 15u, wt = e >> 4;
    const uint32_t zz = ffbh_u32(th);
    const bool has = ((th >> 31) == 0u) & (n1 < room);  // a code starts after the run, before the stop
    const bool table = has & (k != 0u) & (p + n1 + wt <= stop);
    const bool one = has & !table;
    bad = one & (zz >= 16u);
    const bool take1 = one & (zz < 16u);
    p += n1 + (table ? wt : (take1 ? 2u * zz + 1u : 0u));
    return n1 + (table ? k : (take1 ? 1u : 0u));
}
// ... and with the mark pass's one-mark rule (pos_step_lut_mark)
template <int B = kEgLutBits>
__device__ __forceinline__ uint32_t pos_step_lut_mark_bounded(const uint32_t* col, const uint8_t* lut, uint32_t& p,
                                                              bool& bad, uint32_t d0, uint32_t stop) {
    const uint32_t room = stop - p;
    uint32_t hi, lo;
    col_bits64(col, p, hi, lo);
    const uint32_t n1 = __builtin_clz(~hi | (0x80000000u >> min(room, 31u)));
    const uint32_t th = (uint32_t)(((((uint64_t)hi << 32) | lo) << n1) >> 32);
    const uint32_t e = lut[th >> (32 - B)];
    const uint32_t k = e & 15u, wt = e >> 4;
    const uint32_t zz = ffbh_u32(th);
    const bool has = ((th >> 31) == 0u) & (n1 < room);
    const bool full = has & (k != 0u) & (n1 + k <= 32u) & (d0 - n1 - 1u >= k - 1u) & (p + n1 + wt <= stop);
    const bool one = has & !full;
    bad = one & (zz >= 16u);
    const bool take1 = one & (zz < 16u);
    p += n1 + (full ? wt : (take1 ? 2u * zz + 1u : 0u));
    return n1 + (full ? k : (take1 ? 1u : 0u));
}

// Pass-0 / confirming parse of a chunk from chunk-relative bit s to its end (stop = min(512, limit)):
// exactly the codes a one-at-a-time parse reads (every 1-bit code boundary is a code boundary).  The
// interior by table steps without bounds, then the bounded steps to the chunk end, then (only if a long or
// invalid code or the data's end stopped them) the checked steps.  Returns the count; *pos = the exit.
__device__ __forceinline__ uint32_t parse_chunk(const EgDecParams& P, const uint32_t* col, const uint8_t* lut, int64_t b0,
                                                uint32_t s, uint32_t stop, uint32_t limit, uint32_t& pos, bool& invalid) {
    const uint32_t fast_stop = stop > kLeanMargin ? stop - kLeanMargin : 0u;
    // the bounded steps end the parse exactly at the stop -- unless the data ends within reach of the chunk
    // end (a code running past the limit is invalid: the checked steps)
    const uint32_t bstop = limit >= stop + 64u ? stop : 0u;
    uint32_t p = s, n = 0, w_last = 0;
    bool bad = false;
    while (!bad & (p < fast_stop)) n += pos_step_lut(col, lut, p, bad, w_last);
    pos_step_undo(bad, w_last, p, n);
    while (!bad & (p < bstop)) n += pos_step_lut_bounded(col, lut, p, bad, bstop);
    invalid = false;
    if (p < stop) {
        ColReader r{col, &P, (uint64_t)b0, 0, 0, 0, 0, 0};
        r.seek(p);
        while (r.pos < stop && sync_step(r, stop, limit, n, invalid)) {
        }
        p = r.pos;
    }
    pos = p;
    return n;
}

// The resolve walk (pass 0 with resolve, below), chunk-relative: the pass-0 parse of a chunk (a, from its
// first bit) and its true parse (q, from e, the pass-0 exit of the chunk before) are walked until they
// stand on the same bit.  Branch-free steps of the parse behind, read from the column (round 6; rounds 1-5
// took one code per iteration through two buffered readers).  Invariant: every boundary the parse ahead
// visited before its current position lies at or behind the parse behind (it moved only while behind), so
// the next common boundary is at or past `ahead`.  Hence the parse behind may take (a) a run of 1-bit codes
// -- every bit of it a boundary, so a run reaching `ahead` meets there -- and (b) all codes the table sees
// complete when they end at or before `ahead`, else one code.  A code of >= 33 bits or 32 zero bits ends
// the walk unmet (stuck: the confirming parse).
struct Walk {
    uint32_t pa, pq, na, nq;
    bool stuck;
};
__device__ __forceinline__ bool walk_done(const Walk& w, uint32_t limit) {
    return w.pa == w.pq || min(w.pa, w.pq) >= kMeetBits || max(w.pa, w.pq) > limit || w.stuck;
}
// up to `steps` steps (the ended lanes idle); true when the walk has ended
__device__ __forceinline__ bool walk(const uint32_t* col, const uint8_t* lut, uint32_t limit, Walk& w, uint32_t steps) {
    for (uint32_t i = 0; i < steps && !walk_done(w, limit); i++) {
        const bool a_behind = w.pa < w.pq;
        const uint32_t behind = min(w.pa, w.pq), ahead = max(w.pa, w.pq);
        uint32_t hi, lo;
        col_bits64(col, behind, hi, lo);
        const uint32_t n1 = __builtin_clz(~hi | 1u);  // <= 31
        const uint32_t th = (uint32_t)(((((uint64_t)hi << 32) | lo) << n1) >> 32);
        const uint32_t ent = lut[th >> (32 - kEgLutBits)];
        const uint32_t k = ent & 15u, wt = ent >> 4;
        const uint32_t zz = ffbh_u32(th);
        const bool run_meet = behind + n1 >= ahead;
        const bool code = (th >> 31) == 0u;  // a code follows the run (not a capped run)
        const bool table = (k != 0u) & (behind + n1 + wt <= ahead);
        w.stuck = !run_meet & !table & code & (zz >= 16u);
        const uint32_t adv = w.stuck ? 0u : (run_meet ? ahead - behind : n1 + (table ? wt : (code ? 2u * zz + 1u : 0u)));
        const uint32_t cnt = run_meet ? ahead - behind : n1 + (table ? k : (code ? 1u : 0u));
        w.pa += a_behind ? adv : 0u;
        w.na += a_behind && adv ? cnt : 0u;
        w.pq += a_behind ? 0u : adv;
        w.nq += !a_behind && adv ? cnt : 0u;
    }
    return walk_done(w, limit);
}

// The resolve of a block's chunks (every thread calls it: it holds two barriers).  own: the thread's chunk
// is the block's (not the helper, not past the data); e: its true start as far as pass 0 knows it (the
// pass-0 exit of the chunk before, chunk-relative; 0 for chunk 0; ~0u: that parse ended invalid, which a
// confirming pass would repeat from the nominal start: nothing to resolve); x0 / inv0 / n: its pass-0 exit
// and count.  Returns fail (the true exit differs from the pass-0 exit the next chunk was resolved
// against); n / x: the true count and exit (~0u: invalid).
// Walk lengths are short on average but long-tailed (1080p ramp content: mean 1.1 steps, 99th percentile
// 15; the maximum over a wave's 63 chunks averages 15 -- tools/walk_sim.py), and a wave runs as long as its
// longest walk.  So each lane takes kWalkSimt steps, then the walks still going (~10 % on ramp content)
// are queued in LDS and finished by wave 0, 64 at a time: a block pays the long tail once instead of once
// per wave (simulated: 59 -> 26 wave-steps per block on ramp content, 71 -> 30 on uniform noise, with 2
// steps per lane).  Measured (profiles/r06/front/r06_wsimt*): sync pass 280 -> 241 / 246 / 247 us with 2 /
// 4 / 1 steps per lane on ramp content, 824 / 737-744 / 863 us on uniform noise; the queue dealt to all 4
// waves instead of wave 0: 278 / 805 us.  4 steps.
#ifndef DCT3D_WALK_SIMT  // A/B only
#define DCT3D_WALK_SIMT 4
#endif
constexpr uint32_t kWalkSimt = DCT3D_WALK_SIMT;
// qcap: the queue's entries; a walk that finds it full finishes in its own lane (rare: ~10 % of the chunks
// queue, and the sync pass's queue holds 60 of its 255).
__device__ __forceinline__ bool resolve_block(const EgDecParams& P, const uint32_t* win, const uint8_t* lut,
                                              uint32_t* s_q, uint32_t* s_qn, int64_t first, bool own, uint32_t e,
                                              uint32_t x0, bool inv0, uint32_t stop, uint32_t limit, int64_t b0,
                                              uint32_t& n, uint32_t& x, uint32_t qcap = kEgBlock) {
    const uint32_t* col = column(win);
    x = inv0 ? ~0u : x0;
    const bool walking = own && e < kMeetBits;  // (e = ~0u: not walking)
    Walk w{0u, walking ? e : 0u, 0u, 0u, false};
    uint32_t slot = ~0u;
    if (walking && !walk(col, lut, limit, w, kWalkSimt)) {
        slot = atomicAdd(s_qn, 1u);
        if (slot < qcap) {
            s_q[2 * slot] = threadIdx.x | (w.pa << 8) | (w.pq << 16) | (w.na << 24);  // all < 256
            s_q[2 * slot + 1] = w.nq;
        } else {
            (void)walk(col, lut, limit, w, ~0u);
            slot = ~0u;
        }
    }
    __syncthreads();
    const uint32_t qn = min(*s_qn, qcap);
    if (threadIdx.x < 64) {
        for (uint32_t i = threadIdx.x; i < qn; i += 64) {
            const uint32_t a = s_q[2 * i];
            const uint32_t c = a & 255u;
            Walk v{(a >> 8) & 255u, (a >> 16) & 255u, a >> 24, s_q[2 * i + 1], false};
            const int64_t bc = (int64_t)P.start_bit + (first + (int64_t)c) * (int64_t)kChunkBits;
            (void)walk(win + (c >> 5) * (32 * kColW) + (c & 31), lut, rel_bit(P.limit_bit, bc), v, ~0u);
            s_q[2 * i] = c | (v.pa << 8) | (v.pq << 16) | (v.na << 24);
            s_q[2 * i + 1] = v.nq | (v.stuck ? 0x80000000u : 0u);
        }
    }
    __syncthreads();
    if (slot != ~0u) {
        const uint32_t a = s_q[2 * slot], c = s_q[2 * slot + 1];
        w = Walk{(a >> 8) & 255u, (a >> 16) & 255u, a >> 24, c & 0x7FFFFFFFu, (c >> 31) != 0u};
    }
    if (!own || e == ~0u) return false;
    if (walking && w.pa == w.pq && w.pa <= x0) {  // met at or before the pass-0 exit (else: past the data)
        n = n - w.na + w.nq;
        return false;
    }
    // rare (a dense run of long codes): the confirming pass of this chunk, inline
    bool inv2 = false;
    uint32_t x2 = 0;
    n = parse_chunk(P, col, lut, b0, e, stop, limit, x2, inv2);
    x = inv2 ? ~0u : x2;
    // the next chunk was resolved against the pass-0 exit: only a different true exit needs the confirming
    // passes
    return x != (inv0 ? ~0u : x0);
}

// Sync pass.  resolve (pass 0 only): the block owns kEgBlock - 1 chunks, [b * 255, b * 255 + 255), on
// threads 1 .. 255; thread 0 parses chunk b * 255 - 1 (the previous block's last) for its exit only.
// Then, in LDS, chunk t's TRUE parse, from the pass-0 exit e of chunk t - 1 (the first true boundary at
// or past chunk t's start, IF chunk t - 1 is in sync), and chunk t's pass-0 parse, from its start, are
// walked side by side (the one behind advances) until they stand on the same bit: from there both read
// the same codes, so chunk t's pass-0 exit is its true exit and its true count is the pass-0 count,
// minus the pass-0 codes before the meeting point, plus the codes the true parse took to reach it.
// Chunk 0 starts at the true first bit, so when every chunk meets, every exit and count is final by
// induction and no confirming pass is needed; status[0] = 0 says so.  (e = no exit: chunk t - 1's parse
// ended invalid, a confirming pass would restart chunk t at its nominal start, i.e. repeat pass 0: met.)
// A chunk whose parses do not meet within kMeetBits runs its own confirming parse from e through the
// chunk, in place; only if that exit differs from the pass-0 exit (which chunk t + 1 resolved against)
// is status[0] set, and the host then runs confirming passes (iteration 1, plain mapping).  The fused
// front (eg_front_kernel) runs this pass, the scan and the mark pass in one launch; these kernels are its
// non-speculative rerun and the DCT3D_OPT_EG_NO_RESOLVE path.
// DIAG (diagnostic builds, DCT3D_DIAG_FRONT, timing only): 1 = the staging alone, 2 = + the pass-0
// interior loop, 3 = + the whole pass-0 parse, 4 = + the barrier and the exits in LDS, 5 = + the resolve
// walk (no stores); nothing is written
// LDS: table + window + a 60-entry walk queue + 5 words = 23,028 bytes, 7 blocks per CU with 72 VGPRs (the
// pass is latency-bound: 5 blocks instead of 6 cost it 11 %, profiles/r06/front/r06_socc).  The pass-0
// exits reach the next thread by a shuffle, across waves through 4 words.
constexpr uint32_t kSyncQCap = 60;
template <int DIAG>
__device__ __forceinline__ void sync_body(const EgDecParams& P, int iteration, int resolve) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[(kLutBytes + kColBytes) / 4 + 2 * kSyncQCap + 1 + kEgWaves];
    uint8_t* const s_lut = (uint8_t*)lds;
    uint32_t* const win = lds + kLutBytes / 4;
    uint32_t* const s_q = win + kColBytes / 4;  // the resolve's walk queue (resolve_block), its count after it
    uint32_t* const s_qn = s_q + 2 * kSyncQCap;
    uint32_t* const s_xb = s_qn + 1;  // each wave's last pass-0 exit
    copy_lut(s_lut);
    if (threadIdx.x == 0) *s_qn = 0u;
    const bool rs = iteration == 0 && resolve;
    const int64_t b = blockIdx.x;
    const int64_t first = rs ? b * (kEgBlock - 1) - 1 : b * kEgBlock;  // block 0 resolving: chunk -1 (none)
    stage_columns(P, win, first);
    __syncthreads();
    const int64_t ti = first + (int64_t)threadIdx.x;
    const bool live = ti >= 0 && (uint64_t)ti < P.n_chunks;
    const uint64_t t = (uint64_t)ti;
    const int64_t b0 = (int64_t)P.start_bit + ti * (int64_t)kChunkBits;  // absolute bit of the column's bit 0
    const uint32_t limit = rel_bit(P.limit_bit, b0);
    const uint32_t stop = min((uint32_t)kChunkBits, limit);
    const uint32_t* col = column(win);
    if (DIAG == 1) {
        if (col[0] == 0x12345678u && P.n_chunks == 0) P.count[0] = 1u;  // keeps the staging
        return;
    }
    uint32_t s0 = 0;  // iteration 0 (and chunk 0): the chunk's first bit
    if (live && iteration > 0 && t > 0) {
        const uint64_t e = P.exit_in[t - 1];
        s0 = e == kNoExit ? 0u : rel_bit(e, b0);
    }
    uint32_t n = 0, pos = 0;
    bool invalid = false;
    if (DIAG == 2) {
        const uint32_t fast_stop = stop > kLeanMargin ? stop - kLeanMargin : 0u;
        uint32_t p = 0, w_last = 0;
        bool bad = false;
        while (live & !bad & (p < fast_stop)) n += pos_step_lut(col, s_lut, p, bad, w_last);
        if (n == 0xFFFFFFFFu) P.count[0] = p;
        return;
    }
    if (live) n = parse_chunk(P, col, s_lut, b0, s0, stop, limit, pos, invalid);
    if (DIAG == 3) {
        if (n == 0xFFFFFFFFu) P.count[0] = pos;
        return;
    }
    const uint64_t ex = invalid ? kNoExit : (uint64_t)b0 + pos;
    if (!rs) {
        if (!live) return;
        P.exit_out[t] = ex;
        P.count[t] = n;
        if (iteration > 0 && ex != P.exit_in[t]) atomicOr((unsigned int*)&P.status[0], 1u);
        return;
    }
    const uint32_t xv = invalid ? ~0u : pos;
    uint32_t ep = __shfl_up(xv, 1, 64);  // the chunk before's pass-0 exit, in its coordinates
    if ((threadIdx.x & 63) == 63) s_xb[threadIdx.x >> 6] = xv;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) ep = threadIdx.x ? s_xb[(threadIdx.x >> 6) - 1] : ~0u;
    const bool own = live && threadIdx.x > 0;  // thread 0: the helper chunk (written by its owner block)
    // the true start as pass 0 knows it (chunk 0: its first bit)
    const uint32_t e = t == 0 ? 0u : (ep == ~0u ? ~0u : ep - (uint32_t)kChunkBits);
    if (DIAG == 4) {
        if (e == 0x12345678u && n == 0xFFFFFFFFu) P.count[0] = pos;
        return;
    }
    uint32_t x;
    const bool fail = resolve_block(P, win, s_lut, s_q, s_qn, first, own, e, pos, invalid, stop, limit, b0, n, x,
                                    kSyncQCap);
    if (DIAG == 5) {
        if (fail && n == 0xFFFFFFFFu) P.count[0] = x;
        return;
    }
    if (!own) return;
    P.exit_out[t] = x == ~0u ? kNoExit : (uint64_t)b0 + x;
    P.count[t] = n;
    const uint64_t fb = __ballot(fail);
    if (fb != 0ull && (threadIdx.x & 63) == (uint32_t)__builtin_ctzll(fb)) atomicOr((unsigned int*)&P.status[0], 1u);
}
__global__ __launch_bounds__(kEgBlock, 7) void eg_sync_kernel(EgDecParams P, int iteration, int resolve) {
    sync_body<0>(P, iteration, resolve);
}
#ifdef DCT3D_DIAG_FRONT
__global__ __launch_bounds__(kEgBlock) void eg_sync_diag1_kernel(EgDecParams P) { sync_body<1>(P, 0, 1); }
__global__ __launch_bounds__(kEgBlock) void eg_sync_diag2_kernel(EgDecParams P) { sync_body<2>(P, 0, 1); }
__global__ __launch_bounds__(kEgBlock) void eg_sync_diag3_kernel(EgDecParams P) { sync_body<3>(P, 0, 1); }
__global__ __launch_bounds__(kEgBlock) void eg_sync_diag4_kernel(EgDecParams P) { sync_body<4>(P, 0, 1); }
__global__ __launch_bounds__(kEgBlock) void eg_sync_diag5_kernel(EgDecParams P) { sync_body<5>(P, 0, 1); }
#endif

// Decoupled look-back over per-block descriptors (the fused front's chunk value indices):
// desc[b] holds a flag in the top 2 bits -- 1 the block's aggregate, 2 its inclusive prefix, 3 failed --
// and the value below (zeroed by the host before the launch).  Called by a whole wave (64 lanes) of block
// b with the block's aggregate: publishes it, reads the predecessors 64 at a time back to an inclusive
// prefix (waiting for any that has not published), publishes the block's inclusive prefix and returns
// its exclusive one.  Forward progress: a block waits only for lower-numbered blocks, which the dispatcher
// started before it; a wait longer than kLookSpin sleeps (never seen) gives up as failed, and a failed
// block makes every later one fail (the caller then reruns without speculation).
constexpr uint64_t kDescAgg = 1ull << 62, kDescInc = 2ull << 62, kDescFail = 3ull << 62;
constexpr uint64_t kDescVal = (1ull << 62) - 1;
constexpr uint32_t kLookSpin = 1u << 16;
__device__ __forceinline__ uint64_t block_lookback(uint64_t* desc, int64_t b, uint64_t agg, bool& failed) {
    const uint32_t lane = threadIdx.x & 63u;
    uint64_t excl = 0;
    if (b > 0) {
        if (lane == 0)
            __hip_atomic_store(&desc[b], failed ? kDescFail : (kDescAgg | agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        int64_t look = b - 1;
        uint32_t spins = 0;
        while (!failed) {
            const int64_t i = look - (int64_t)lane;
            const uint64_t d = i >= 0 ? __hip_atomic_load(&desc[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                      : kDescInc;  // before block 0: an inclusive prefix of 0
            const uint32_t flag = (uint32_t)(d >> 62);
            const uint64_t stopm = __ballot(flag >= 2u);  // an inclusive prefix or a failure
            const uint32_t s = stopm ? (uint32_t)__builtin_ctzll(stopm) : 64u;
            const uint64_t upto = s >= 63u ? ~0ull : (2ull << s) - 1ull;  // lanes 0 .. s
            if ((__ballot(flag == 0u) & upto) != 0ull) {  // a predecessor not published yet: wait
                if (++spins > kLookSpin) failed = true;
                __builtin_amdgcn_s_sleep(4);
                continue;
            }
            if (s < 64u && __shfl(flag, s, 64) == 3u) {
                failed = true;
                break;
            }
            uint64_t v = lane <= s ? (d & kDescVal) : 0ull;
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
            excl += v;
            if (s < 64u) break;
            look -= 64;
        }
    }
    if (lane == 0)
        __hip_atomic_store(&desc[b], failed ? kDescFail : (kDescInc | (excl + agg)), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    return excl;
}

// The mark parse of one chunk from its true start sp (chunk-relative) with its first value idx0: the bit
// position of every 32nd value.  The marks are collected in the thread's slots myk[SS * k] (2 bytes each,
// relative to the true start) and written out at the end, each thread its consecutive marks back to back, so that the L2 assembles whole
// lines (round 4: WRITE_SIZE 1.67 -> 0.52 GB, the pass 708 -> 529 us; stored one at a time as the parse
// reached them the lines were written back partial).  Marks leave as the low 16 bits of their bit position
// (round 5), the whole position of every 64th (a consumer group's first) in mark_base (mark_offset).
// Every step of the interior loops stores its mark candidate to the current slot, and a hit moves on to the
// next (no branch): a step without a mark leaves a value in the slot after the last mark, which the next
// mark overwrites or nobody reads -- kMkSlot entries: 16 marks (a chunk's true parse takes <= 512 values)
// and that one.
// Slot layout (round 6): mark k of a chunk lives in word k - kMkPad of the chunk's own column (SS = 64:
// 128 bytes per slot, the column's stride), the first kMkPad in words in front of the column.  A column word
// is dead once the parse has passed it: mark k sits at value >= 32 k of the chunk, so at bit >= 32 k, and
// slot k is written only after mark k - 1 (bit >= 32 (k - 1)) -- from then on the steps use words >=
// k - 1 (col_bits64 also reads word p / 32 - 1 at p = 0 mod 32, and ignores it; the checked reader and
// the undo of a long code never go below the last mark), above word k - kMkPad.  So the pass needs no LDS
// of its own for the marks: 24.6 instead of 31.3 KB per block, 6 blocks per CU instead of 5.
constexpr uint32_t kMkSlot = 17;
constexpr uint32_t kMkPad = 2;
#ifndef DCT3D_MARK_LUT_BITS  // A/B only: the mark pass's table width
#define DCT3D_MARK_LUT_BITS 12
#endif
constexpr int kMarkLutBits = DCT3D_MARK_LUT_BITS;
template <bool WRITE = true, uint32_t SS = 1, int LB = kEgLutBits>
__device__ __forceinline__ void mark_chunk(const EgDecParams& P, const uint32_t* col, const uint8_t* lut, uint16_t* myk,
                                           int64_t b0, uint32_t sp, uint64_t idx0) {
    const uint32_t end = (uint32_t)kChunkBits;
    const uint32_t limit = rel_bit(P.limit_bit, b0);
    // chunk-relative 32-bit value count i (value idx0 + i): the 64-bit index arithmetic per step was a
    // large part of the pass.  A chunk holds at most ~kChunkBits + 64 codes, so rem below never binds
    // unless the wanted values end inside this chunk.
    const uint64_t rem64 = P.n_values - idx0;
    const uint32_t rem = (uint32_t)min(rem64, (uint64_t)(2 * kChunkBits));
    const bool ends_here = rem64 <= 2 * kChunkBits;
    const uint32_t ph = (uint32_t)idx0 & (kMarkVals - 1);
    const uint32_t sh = ph ? 1u : 0u;       // slot of value j: (ph + j) / 32 - sh (16 slots)
    const uint64_t gm0 = idx0 / kMarkVals;  // mark gm0 + k = mark of value idx0 + 32 k - ph
    uint32_t i = 0, code;
    // Interior of the chunk: a step moves at most 31 + 31 bits and 32 values, so while the parse is
    // kLeanMargin bits short of the chunk end and of the data limit none of the bounds below can bind -- a
    // lean loop without them (a long or invalid code leaves it for the checked loop, which reads or reports
    // it).  The lean loops run only in chunks that cannot hold the last wanted value (rem64 > 2 kChunkBits;
    // the few others take the checked steps whole): there the value count never binds, and the loops test
    // only the position.
    const uint32_t lim_end = ends_here ? 0u : min(end, limit);
    const uint32_t fast_end = lim_end > kLeanMargin ? lim_end - kLeanMargin : 0u;
    uint32_t p = sp;
    {
        bool bad = false;
        // the next mark: chunk-relative value index nm (value idx0 + nm), its slot mp; a step takes nv <= 32
        // values, so at most one mark, value d0 = nm - i of the step
        uint32_t nm = (0u - ph) & (kMarkVals - 1);
        uint16_t* mp = myk;
        auto mark = [&](uint32_t at, uint32_t nv, uint32_t d0) {
            const bool hit = d0 < nv;
            *mp = (uint16_t)(at - sp);  // no branch: a miss is overwritten by the next mark or never read
            nm += hit ? kMarkVals : 0u;
            mp += hit ? SS : 0u;
            i += nv;
        };
        // table steps that stop on the mark (nv <= 32): the mark is value d0 of the step, at bit p0 + d0
        uint32_t w_last = 0;
        while (!bad & (p < fast_end)) {
            const uint32_t p0 = p;
            const uint32_t d0 = nm - i;
            mark(p0 + d0, pos_step_lut_mark<LB>(col, lut, p, bad, d0, w_last), d0);
        }
        // the long or invalid code the last step met (its mark, if it is one, was stored at its first bit:
        // the checked loop stores the same or ends the pass)
        pos_step_undo(bad, w_last, p, i);
        // to the chunk end exactly (as the sync pass; the chunk holding the last wanted value and the data's
        // end take the checked steps)
        const uint32_t bend = limit >= end + 64u && !ends_here ? end : 0u;
        while (!bad & (p < bend)) {
            const uint32_t p0 = p;
            const uint32_t d0 = nm - i;
            mark(p0 + d0, pos_step_lut_mark_bounded<LB>(col, lut, p, bad, d0, bend), d0);
        }
    }
    if (i < rem && p < end) {
        ColReader r{col, &P, (uint64_t)b0, 0, 0, 0, 0, 0};
        r.seek(p);
        while (i < rem && r.pos < end) {
            const uint32_t p0 = r.pos;
            if (p0 >= limit) {  // ran out of bits
                atomicOr((unsigned int*)&P.status[2], 2u);
                return;
            }
            // one step = a run of 1-bit codes, then one longer code (as sync_step)
            const uint32_t room = min(min(end - p0, limit - p0), rem - i);
            const uint32_t k = r.ones(min(room, 64u));
            if (k) {  // values i .. i + k - 1 are zeros at bits p0 .. p0 + k - 1
                for (uint32_t j = ((ph + i + kMarkVals - 1) & ~(kMarkVals - 1)) - ph; j < i + k; j += kMarkVals)
                    myk[SS * ((ph + j) / kMarkVals - sh)] = (uint16_t)(p0 + (j - i) - sp);
                i += k;
                if (ends_here && i == rem) P.status[1] = (uint64_t)b0 + r.pos;  // the bit after the last wanted value
            }
            // the run ended the chunk or the wanted values, or the buffered bits ran out inside it (refill)
            if (i >= rem || r.pos >= end || !r.at_long_code()) continue;
            const uint32_t p1 = r.pos;
            if (!r.get(code) || r.pos > limit) {
                // ran out of bits (2) unless 32 zero bits lie inside the data (corrupt, 1)
                atomicOr((unsigned int*)&P.status[2], (uint64_t)p1 + 32 <= limit && r.pos <= limit ? 1u : 2u);
                return;
            }
            // a code of 33+ bits (|v| >= 2^15): the consumers' parse steps check for them (parse_step CHECK).
            // Every code of the wanted values is parsed here or in the lean loops above, which leave every
            // such code to this loop.
            if (code >= 0x10000u) atomicOr((unsigned int*)&P.status[3], 1u);
            if (((ph + i) & (kMarkVals - 1)) == 0) myk[SS * ((ph + i) / kMarkVals - sh)] = (uint16_t)(p1 - sp);
            if (++i == rem && ends_here) P.status[1] = (uint64_t)b0 + r.pos;
        }
    }
    if (!WRITE) {  // diagnostic
        if (i == 0xFFFFFFFFu) P.mark[0] = (uint16_t)p;
        return;
    }
    // the chunk's marks k = sh .. (ph + i - 1) / 32, back to back
    const uint64_t a0 = (uint64_t)b0 + sp;
    uint16_t* const mk = P.mark + gm0;
    for (uint32_t k = sh; k < (ph + i + kMarkVals - 1) / kMarkVals; k++) {
        const uint64_t m = a0 + myk[SS * (k - sh)];
        mk[k] = (uint16_t)m;
        if (((gm0 + k) & (kMarkGroup - 1)) == 0) P.mark_base[(gm0 + k) / kMarkGroup] = m;
    }
}

// Mark pass (the non-speculative path): each chunk parsed once more from its true start (the converged
// exit of the chunk before), its first value index from the scan.
template <int DIAG>
__device__ __forceinline__ void mark_body(const EgDecParams& P) {
    constexpr uint32_t kWinWords = kEgBlock * (kColW + kMkPad);  // the columns with the marks' pad
    constexpr uint32_t kMLut = 1u << kMarkLutBits;
    __shared__ __attribute__((aligned(16))) uint32_t lds[kMLut / 4 + kWinWords + kEgWaves + 1];
    uint8_t* const s_lut = (uint8_t*)lds;
    uint32_t* const win = lds + kMLut / 4;
    uint32_t* const s_ws = win + kWinWords;  // the waves' count sums, then the parts' sum
    copy_lut<kMarkLutBits>(s_lut);
    // the sync pass's verdict: status[0] != 0 only after a speculative pass 0 whose chunks did not all
    // resolve (the converged confirming passes leave it 0): no marks, the consumers skip themselves
    if (P.status[0] != 0) {  // grid-uniform
        if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr((unsigned int*)&P.status[2], 4u);
        return;
    }
    const int64_t first = (int64_t)blockIdx.x * kEgBlock;
    const uint64_t t = (uint64_t)first + threadIdx.x;
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    // the chunk's count and true start, and wave 0's parts of the chunks before the block within its 4,096
    // (eg_dscan_reduce_kernel), in flight together at the top issue priority with the window's loads
    __builtin_amdgcn_s_setprio(3);
    const uint32_t cnt = t < P.n_chunks ? P.count[t] : 0u;
    const uint64_t s = t == 0 ? P.start_bit : (t < P.n_chunks ? P.exit_in[t - 1] : kNoExit);  // the converged exits
    const uint32_t pj = (uint32_t)(blockIdx.x & 15u);
    const uint32_t pv = (wave == 0 && lane < pj) ? P.part[(uint64_t)blockIdx.x - pj + lane] : 0u;
    const uint64_t bb = P.bsum[blockIdx.x >> 4];
    __builtin_amdgcn_s_setprio(0);
    stage_columns<kMkPad>(P, win, first);
    // the block's exclusive scan of the counts: in the wave by shuffles, across the waves through LDS
    uint32_t incl = cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t v = __shfl_up(incl, o, 64);
        if (lane >= (uint32_t)o) incl += v;
    }
    if (lane == 63) s_ws[wave] = incl;
    if (wave == 0) {
        uint32_t ps = pv;
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) ps += __shfl_xor(ps, o, 64);
        if (lane == 0) s_ws[kEgWaves] = ps;
    }
    __syncthreads();
    if (DIAG == 1) {
        if (column<kMkPad>(win)[0] == 0x12345678u && P.n_chunks == 0) P.count[0] = 1u;  // keeps the staging
        return;
    }
    if (t >= P.n_chunks) return;
    uint64_t idx0 = bb + s_ws[kEgWaves] + (incl - cnt);
#pragma unroll
    for (uint32_t w = 0; w < (uint32_t)kEgWaves; w++) idx0 += w < wave ? s_ws[w] : 0u;
    // (Round 6: the value index by a look-back over the chunk counts instead of the scan ran the pass
    // 295 -> 440 us, profiles/r06/front/r06_mlb: an uncached round trip on every block's critical path.)
    if (idx0 >= P.n_values) return;
    if (s == kNoExit) return;  // the true parse stopped in an earlier chunk: reported by that chunk
    const int64_t b0 = (int64_t)P.start_bit + (int64_t)t * (int64_t)kChunkBits;
    uint32_t* const col = column<kMkPad>(win);
    mark_chunk<DIAG == 0, 64, kMarkLutBits>(P, col, s_lut, (uint16_t*)(col - 32 * kMkPad), b0, rel_bit(s, b0), idx0);
}
__global__ __launch_bounds__(kEgBlock) void eg_mark_kernel(EgDecParams P) { mark_body<0>(P); }
#ifdef DCT3D_DIAG_FRONT
__global__ __launch_bounds__(kEgBlock) void eg_mark_diag1_kernel(EgDecParams P) { mark_body<1>(P); }
__global__ __launch_bounds__(kEgBlock) void eg_mark_diag2_kernel(EgDecParams P) { mark_body<2>(P); }
#endif

// The fused front (round 6): the resolving sync pass, the scan of the chunk counts and the mark pass in
// one launch, the stream staged into LDS once.  Block b: pass 0 and the resolve walk of its 255 chunks (as
// eg_sync_kernel), a block scan of their true counts, then the counts of every earlier block by a
// decoupled look-back over per-block descriptors (desc[b]: flag in the top 2 bits -- 1 aggregate, 2
// inclusive prefix, 3 failed -- the value below; zeroed by the host before the launch), then the mark
// parse of each chunk from its true start (the pass-0 exit of the chunk before, in LDS).  Forward progress:
// a block only waits for lower-numbered blocks, which the dispatcher started before it; a wait longer than
// kLookSpin sleeps (never seen) gives up as failed.  A failed block (a chunk that did not resolve, or the
// wait) makes every later block fail too: no marks there, status[0] and status[2] bit 4 set, the consumer
// skips itself and the host reruns the non-speculative front (eg_sync_kernel passes, scan, eg_mark_kernel).
// Replaces: sync pass 0 (its window staging), the three scan launches, the mark pass's window staging and
// its reads of the chunk offsets and exits.
__global__ __launch_bounds__(kEgBlock) void eg_front_kernel(EgDecParams P, uint64_t* desc, int force_fail) {
    __shared__ __attribute__((aligned(16)))
    uint32_t lds[(kLutBytes + kColBytes) / 4 + kEgBlock + kEgBlock * kMkSlot / 2 + kEgWaves + 6];
    static_assert(kEgBlock * kMkSlot / 2 >= 2 * kEgBlock, "the walk queue fits the mark slots");
    uint8_t* const s_lut = (uint8_t*)lds;
    uint32_t* const win = lds + kLutBytes / 4;
    uint32_t* const s_exit = win + kColBytes / 4;
    uint16_t* const s_mk = (uint16_t*)(s_exit + kEgBlock);
    uint32_t* const s_wsum = s_exit + kEgBlock + kEgBlock * kMkSlot / 2;  // per-wave count sums
    uint64_t* const s_misc = (uint64_t*)(s_wsum + kEgWaves);             // [0] prefix, [1] failed
    uint32_t* const s_qn = (uint32_t*)(s_misc + 2);
    uint32_t* const s_q = (uint32_t*)s_mk;  // the resolve's walk queue, before the mark slots are used
    copy_lut(s_lut);
    if (threadIdx.x == 0) *s_qn = 0u;
    const int64_t b = blockIdx.x;
    const int64_t first = b * (kEgBlock - 1) - 1;
    stage_columns(P, win, first);
    __syncthreads();
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t ti = first + (int64_t)tid;
    const bool live = ti >= 0 && (uint64_t)ti < P.n_chunks;
    const uint64_t t = (uint64_t)ti;
    const int64_t b0 = (int64_t)P.start_bit + ti * (int64_t)kChunkBits;
    const uint32_t limit = rel_bit(P.limit_bit, b0);
    const uint32_t stop = min((uint32_t)kChunkBits, limit);
    const uint32_t* col = column(win);
    // pass 0 from the chunk's first bit
    uint32_t n = 0, pos = 0;
    bool invalid = false;
    if (live) n = parse_chunk(P, col, s_lut, b0, 0u, stop, limit, pos, invalid);
    s_exit[tid] = invalid ? ~0u : pos;
    __syncthreads();
    // the resolve: the true count and the true start (the pass-0 exit of the chunk before, which the walk
    // proves true unless it fails) of each owned chunk (threads 1 .. 255)
    const bool own = live && tid > 0;
    const uint32_t ep = tid ? s_exit[tid - 1] : ~0u;
    const uint32_t sp = t == 0 ? 0u : (ep == ~0u ? ~0u : ep - (uint32_t)kChunkBits);
    uint32_t cnt = n, x;
    const bool fail = resolve_block(P, win, s_lut, s_q, s_qn, first, own, sp, pos, invalid, stop, limit, b0, cnt, x);
    if (!own) cnt = 0;
    // block scan of the counts (the helper's is 0): in the wave by shuffles, across the 4 waves in LDS
    uint32_t incl = cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t v = __shfl_up(incl, o, 64);
        if (lane >= (uint32_t)o) incl += v;
    }
    if (lane == 63) s_wsum[wave] = incl;
    const bool wfail = __ballot(fail) != 0ull;
    if (tid == 0) s_misc[1] = 0;
    __syncthreads();
    if ((wfail || force_fail) && lane == 0) atomicOr((unsigned int*)&s_misc[1], 1u);
    uint64_t wpre = 0, agg = 0;
#pragma unroll
    for (uint32_t w = 0; w < (uint32_t)kEgWaves; w++) {
        wpre += w < wave ? s_wsum[w] : 0u;
        agg += s_wsum[w];
    }
    __syncthreads();
    // the look-back (wave 0): the counts of every chunk before the block's first
    if (wave == 0) {
        bool failed = s_misc[1] != 0;
        const uint64_t excl = block_lookback(desc, b, agg, failed);
        if (lane == 0) {
            s_misc[0] = excl;
            s_misc[1] = failed ? 1u : 0u;
            // the total count (the scan's, status[4]: fewer values than wanted is ENODATA)
            if (!failed && b == (int64_t)gridDim.x - 1) P.status[4] = excl + agg;
        }
    }
    __syncthreads();
    if (s_misc[1] != 0) {  // block-uniform: rerun without speculation
        if (tid == 0) {
            atomicOr((unsigned int*)&P.status[0], 1u);
            atomicOr((unsigned int*)&P.status[2], 4u);
        }
        return;
    }
    if (!own || sp == ~0u) return;  // sp = ~0u: the true parse stopped in an earlier chunk (reported there)
    const uint64_t idx0 = s_misc[0] + wpre + (incl - cnt);
    if (idx0 >= P.n_values) return;
    mark_chunk(P, col, s_lut, s_mk + tid * kMkSlot, b0, sp, idx0);
}

template <int D>
__global__ __launch_bounds__(kEgBlock) void eg_emit_kernel(EgDecParams P) {
    constexpr uint32_t CS = 64 * D, PARTS = CS / kMarkVals, CPW = 64 / PARTS;
    static_assert(CPW * CS * 4 == kEmitWinWords * 4, "one wave's cubes fill its staging");
    __shared__ uint32_t lds[kEgWaves][kEmitWinWords];
    __shared__ uint16_t s_diag[CS];
    if (P.status[2] != 0) return;  // corrupt / short stream: reported, nothing written (block-uniform)
    for (uint32_t i = threadIdx.x; i < CS; i += kEgBlock) s_diag[i] = P.diag[i];
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t n_marks = P.n_values / kMarkVals;
    const uint64_t m0 = ((uint64_t)blockIdx.x * kEgWaves + wave) * 64;
    if (m0 >= n_marks) return;
    const bool lv = m0 + lane < n_marks;
    static_assert(kMarkGroup == 64, "a wave = one mark group");
    const uint64_t gb = P.mark_base[m0 / kMarkGroup];  // wave-uniform
    const uint64_t first = gb;
    const uint64_t last = m0 + 64 < n_marks ? P.mark_base[m0 / kMarkGroup + 1] : P.status[1];  // wave-uniform
    const uint32_t off = mark_offset(lv ? P.mark[m0 + lane] : 0u, (uint16_t)gb);
    const uint64_t my = lv ? gb + off : 0;
    const uint64_t w0 = first >> 5;
    const uint64_t span = (last >> 5) + 5 - w0;  // + 5 words of slack: parse_win
    const bool fits = span <= kEmitWinWords - 1;  // wave-uniform
    const uint32_t nwin = (uint32_t)(fits ? span : 0);
    uint32_t* wl = lds[wave];
    uint32_t* win = wl + 1;  // the window one word into the region: parse_step reads win[-1]
    // 4 loads in flight per lane before the LDS writes (as decode_eg_kernel's staging)
    const uint32_t nst = P.n_words ? nwin : 0u;  // (an empty stream: reported by the mark pass)
    for (uint32_t i0 = 0; i0 < nst; i0 += 256) {
        uint32_t t[4];
#pragma unroll
        for (int b = 0; b < 4; b++) t[b] = P.words[min(w0 + i0 + b * 64 + lane, P.n_words - 1)];
#pragma unroll
        for (int b = 0; b < 4; b++) {
            const uint32_t i = i0 + b * 64 + lane;
            if (i < nwin) win[i] = w0 + i < P.n_words ? __builtin_bswap32(t[b]) : 0u;
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    uint32_t v[kMarkVals];
    parse_codes<kMarkVals>(P, win, nwin, w0, fits, P.status[3] != 0,
                           my > w0 * 32 ? (uint32_t)min(my - w0 * 32, (uint64_t)0xFFFFFFFFu) : 0u, v);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint32_t c = lane / PARTS, part = lane % PARTS;
    int32_t* st = (int32_t*)wl + c * CS;
#pragma unroll
    for (uint32_t i = 0; i < kMarkVals; i++) st[s_diag[part * kMarkVals + i]] = eg_value_fast(v[i]);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    int32_t* q = P.q + m0 * kMarkVals;  // value index of the wave's first cube
    const uint64_t nv = P.n_values - m0 * kMarkVals;
#pragma unroll
    for (uint32_t t = 0; t < 8; t++) {
        const uint32_t e = (t * 64 + lane) * 4;
        if (e < nv) *(int4*)(q + e) = *(const int4*)((const int32_t*)wl + e);
    }
}

}  // namespace

int launch_eg_encode(int D, const EgParams& P, hipStream_t st) {
    if (P.n_cubes == 0) return 0;
    const uint64_t cube_blocks = (P.n_cubes + kEgWaves - 1) / kEgWaves;
    const uint64_t n_chunks = (P.n_cubes + kScanChunk - 1) / kScanChunk;
    if (cube_blocks > 0x7FFFFFFFull) return -1;
    if (D == 8) hipLaunchKernelGGL(eg_len_kernel<8>, dim3((uint32_t)cube_blocks), dim3(kEgBlock), 0, st, P);
    else hipLaunchKernelGGL(eg_len_kernel<4>, dim3((uint32_t)cube_blocks), dim3(kEgBlock), 0, st, P);
    hipLaunchKernelGGL(eg_scan_reduce_kernel, dim3((uint32_t)n_chunks), dim3(kEgBlock), 0, st, P);
    hipLaunchKernelGGL(eg_scan_top_kernel, dim3(1), dim3(1024), 0, st, P, (uint32_t)n_chunks);
    hipLaunchKernelGGL(eg_scan_apply_kernel, dim3((uint32_t)n_chunks), dim3(kEgBlock), 0, st, P);
    static int wgrid = -1;
    if (wgrid < 0) {  // persistent-style writer: 8 blocks (32 waves) per CU
        int dev = 0, cus = 256;
        if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        wgrid = cus * 8;
    }
    const uint32_t wblocks = (uint32_t)(cube_blocks < (uint64_t)wgrid ? cube_blocks : (uint64_t)wgrid);
    if (D == 8) hipLaunchKernelGGL(eg_write_kernel<8>, dim3(wblocks), dim3(kEgBlock), 0, st, P);
    else hipLaunchKernelGGL(eg_write_kernel<4>, dim3(wblocks), dim3(kEgBlock), 0, st, P);
    hipLaunchKernelGGL(eg_stitch_kernel, dim3((uint32_t)((P.n_cubes + kEgBlock - 1) / kEgBlock)), dim3(kEgBlock), 0, st, P);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace dct3d

namespace dct3d {

int launch_eg_sync(const EgDecParams& P, int iteration, int resolve, hipStream_t st) {
    if (P.n_chunks == 0) return 0;
    const bool rs = iteration == 0 && resolve;
    const uint64_t per = rs ? kEgBlock - 1 : kEgBlock;
#ifdef DCT3D_DIAG_FRONT  // diagnostic build: the resolving pass's parts before it (timing only)
    if (rs) {
        const dim3 g((uint32_t)((P.n_chunks + per - 1) / per));
        hipLaunchKernelGGL(eg_sync_diag1_kernel, g, dim3(kEgBlock), 0, st, P);
        hipLaunchKernelGGL(eg_sync_diag2_kernel, g, dim3(kEgBlock), 0, st, P);
        hipLaunchKernelGGL(eg_sync_diag3_kernel, g, dim3(kEgBlock), 0, st, P);
        hipLaunchKernelGGL(eg_sync_diag4_kernel, g, dim3(kEgBlock), 0, st, P);
        hipLaunchKernelGGL(eg_sync_diag5_kernel, g, dim3(kEgBlock), 0, st, P);
    }
#endif
    hipLaunchKernelGGL(eg_sync_kernel, dim3((uint32_t)((P.n_chunks + per - 1) / per)), dim3(kEgBlock), 0, st, P,
                       iteration, (int)rs);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_eg_scan(const EgParams& P, hipStream_t st) {
    if (P.n_cubes == 0) return 0;
    const uint64_t n_chunks = (P.n_cubes + kScanChunk - 1) / kScanChunk;
    hipLaunchKernelGGL(eg_scan_reduce_kernel, dim3((uint32_t)n_chunks), dim3(kEgBlock), 0, st, P);
    hipLaunchKernelGGL(eg_scan_top_kernel, dim3(1), dim3(1024), 0, st, P, (uint32_t)n_chunks);
    hipLaunchKernelGGL(eg_scan_apply_kernel, dim3((uint32_t)n_chunks), dim3(kEgBlock), 0, st, P);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_eg_compact(const EgParams& P, const uint32_t* slot, uint32_t seg_cap, hipStream_t st) {
    if (P.n_cubes == 0) return 0;
    if (launch_eg_scan(P, st)) return -1;
    const uint64_t per = (uint64_t)kEgWaves * kCompactSPW;
    const uint64_t blocks = (P.n_cubes + per - 1) / per;
    hipLaunchKernelGGL(eg_compact_kernel, dim3((uint32_t)blocks), dim3(kEgBlock), 0, st, P, slot, seg_cap);
    hipLaunchKernelGGL(eg_stitch_kernel, dim3((uint32_t)((P.n_cubes + kEgBlock - 1) / kEgBlock)), dim3(kEgBlock), 0, st, P);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_eg_stitch(const EgParams& P, hipStream_t st) {
    if (P.n_cubes == 0) return 0;
    hipLaunchKernelGGL(eg_stitch_kernel, dim3((uint32_t)((P.n_cubes + kEgBlock - 1) / kEgBlock)), dim3(kEgBlock), 0, st, P);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// desc: one zeroed word per block (front_blocks); force_fail (test option): every block fails
uint64_t front_blocks(uint64_t n_chunks) { return (n_chunks + kEgBlock - 2) / (kEgBlock - 1); }
int launch_eg_front(const EgDecParams& P, uint64_t* desc, int force_fail, hipStream_t st) {
    if (P.n_chunks == 0) return 0;
    const uint64_t blocks = front_blocks(P.n_chunks);
    if (blocks > 0x7FFFFFFFull) return -1;
    hipLaunchKernelGGL(eg_front_kernel, dim3((uint32_t)blocks), dim3(kEgBlock), 0, st, P, desc, force_fail);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_eg_dscan(const EgDecParams& P, const EgParams& S, hipStream_t st) {
    if (P.n_chunks == 0) return 0;
    const uint64_t nb = (P.n_chunks + kScanChunk - 1) / kScanChunk;
    hipLaunchKernelGGL(eg_dscan_reduce_kernel, dim3((uint32_t)nb), dim3(kEgBlock), 0, st, P);
    hipLaunchKernelGGL(eg_scan_top_kernel, dim3(1), dim3(1024), 0, st, S, (uint32_t)nb);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
int launch_eg_mark(const EgDecParams& P, hipStream_t st) {
    if (P.n_chunks == 0) return 0;
#ifdef DCT3D_DIAG_FRONT  // diagnostic build: the mark pass's parts before it (timing only)
    hipLaunchKernelGGL(eg_mark_diag1_kernel, dim3((uint32_t)((P.n_chunks + kEgBlock - 1) / kEgBlock)), dim3(kEgBlock), 0, st, P);
    hipLaunchKernelGGL(eg_mark_diag2_kernel, dim3((uint32_t)((P.n_chunks + kEgBlock - 1) / kEgBlock)), dim3(kEgBlock), 0, st, P);
#endif
    hipLaunchKernelGGL(eg_mark_kernel, dim3((uint32_t)((P.n_chunks + kEgBlock - 1) / kEgBlock)), dim3(kEgBlock), 0, st, P);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_eg_emit(int D, const EgDecParams& P, hipStream_t st) {
    const uint64_t waves = (P.n_values / kMarkVals + 63) / 64;
    if (waves == 0) return 0;
    const uint32_t blocks = (uint32_t)((waves + kEgWaves - 1) / kEgWaves);
    if (D == 8) hipLaunchKernelGGL(eg_emit_kernel<8>, dim3(blocks), dim3(kEgBlock), 0, st, P);
    else hipLaunchKernelGGL(eg_emit_kernel<4>, dim3(blocks), dim3(kEgBlock), 0, st, P);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_eg_decode_write(int D, const EgDecParams& P, hipStream_t st) {
    if (launch_eg_mark(P, st)) return -1;
    return launch_eg_emit(D, P, st);
}

}  // namespace dct3d
