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

// one block: exclusive scan of the chunk sums (offset by the carried bits), total, capacity check
__global__ __launch_bounds__(1024) void eg_scan_top_kernel(EgParams P, uint32_t n_chunks) {
    __shared__ uint64_t buf[1024];
    uint64_t carry = P.carry_bits;
    for (uint32_t c0 = 0; c0 < n_chunks; c0 += 1024) {
        const uint32_t i = c0 + threadIdx.x;
        const uint64_t v = i < n_chunks ? P.bsum[i] : 0;
        buf[threadIdx.x] = v;
        __syncthreads();
        for (int o = 1; o < 1024; o <<= 1) {  // Hillis-Steele inclusive scan
            const uint64_t t = threadIdx.x >= (unsigned)o ? buf[threadIdx.x - o] : 0;
            __syncthreads();
            buf[threadIdx.x] += t;
            __syncthreads();
        }
        if (i < n_chunks) P.bsum[i] = carry + buf[threadIdx.x] - v;
        carry += buf[1023];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        P.status[0] = carry;  // total bits including the carried ones
        if ((carry + 31) / 32 > P.out_cap_words) atomicOr((unsigned int*)&P.status[1], 1u);
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
// a block's window: its 256 chunks plus slack (a parse ends < 27 bits past its chunk; the reader's
// buffer and the long-code path look < 96 bits ahead of its position); behind it the mark pass's dummies
// (eg_mark_kernel: 2 bytes per thread)
constexpr uint32_t kSyncWinWords = kEgBlock * (uint32_t)(kChunkBits / 32) + 8;
constexpr uint32_t kSyncWinAlloc = kSyncWinWords + kEgBlock / 2;
static_assert(kChunkBits == 512 && kEgBlock == 256, "16-word chunks");
constexpr uint32_t kMarkVals = 32;          // values per emit lane / per mark
constexpr uint32_t kEmitWinWords = 2048;    // per wave: window (<= 2,048 values x 27 bits) / 8 KiB staging

__device__ __forceinline__ uint64_t chunk_start(const EgDecParams& P, uint64_t t, int iteration) {
    if (t == 0) return P.start_bit;
    if (iteration == 0) return P.start_bit + t * kChunkBits;
    const uint64_t e = P.exit_in[t - 1];
    return e == kNoExit ? P.start_bit + t * kChunkBits : e;
}

// The block's window (chunks [first, first + kEgBlock) and 8 slack words), then a barrier.  Thread t
// loads its own chunk's 16 words as four 16-byte loads (all in flight at once) and writes word j of it to
// LDS as four 16-byte stores.  (Rounds 1-4: 17 coalesced dword loads per thread, thread i storing word
// i + 256 b: the four 16-byte loads made the sync pass 422 -> 405 us, the mark pass 489 -> 471 us.)
// Threads 0 and 1 also take the slack chunk's two quarters.  The data's last window (zeros past the
// end) takes single predicated loads.
__device__ __forceinline__ LdsBits stage_block_window(const EgDecParams& P, uint32_t* win, uint64_t first) {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4), aligned(4)));
    const uint64_t w0 = (P.start_bit + first * kChunkBits) >> 5;
    const uint32_t t = threadIdx.x;
    const bool slack = t < 2;  // quarter t of the slack chunk (kEgBlock)
    u32x4 v[5];
    if (w0 + kSyncWinWords <= P.n_words) {  // block-uniform
        const uint32_t* src = P.words + w0;
#pragma unroll
        for (uint32_t q = 0; q < 4; q++) v[q] = *(const u32x4*)(src + 16 * t + 4 * q);
        v[4] = slack ? *(const u32x4*)(src + 16 * kEgBlock + 4 * t) : u32x4{0u, 0u, 0u, 0u};
    } else {
#pragma unroll
        for (uint32_t q = 0; q < 5; q++) {
            const uint64_t k0 = w0 + (q < 4 ? 16 * t + 4 * q : 16 * kEgBlock + 4 * t);
#pragma unroll
            for (uint32_t e = 0; e < 4; e++)
                v[q][e] = k0 + e < P.n_words && (q < 4 || slack) ? P.words[k0 + e] : 0u;
        }
    }
#pragma unroll
    for (uint32_t q = 0; q < 4; q++)
        *(uint4*)(win + 16 * t + 4 * q) = make_uint4(__builtin_bswap32(v[q][0]), __builtin_bswap32(v[q][1]),
                                                     __builtin_bswap32(v[q][2]), __builtin_bswap32(v[q][3]));
    if (slack)
        *(uint4*)(win + 16 * kEgBlock + 4 * t) = make_uint4(__builtin_bswap32(v[4][0]), __builtin_bswap32(v[4][1]),
                                                            __builtin_bswap32(v[4][2]), __builtin_bswap32(v[4][3]));
    __syncthreads();
    return LdsBits{win, w0, kSyncWinWords};
}
__device__ __forceinline__ LdsBits stage_block_window(const EgDecParams& P, uint32_t* win) {
    return stage_block_window(P, win, (uint64_t)blockIdx.x * kEgBlock);
}

// window-relative form of an absolute bit position (clamped: positions past the window behave as the
// window's end, which only a limit or end beyond the window ever is)
__device__ __forceinline__ uint32_t rel_bit(uint64_t p, uint64_t base) {
    return p <= base ? 0u : (p - base >= 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)(p - base));
}

// A parse from a wrong start meets the true parse (a boundary of both) within 90 bits on every one of
// 10.7 k chunks of the 1080p content (within 64 bits on 99.57 %, at the chunk start on half of them).
constexpr uint32_t kMeetBits = 128;

// One parse step (a run of 1-bit codes, or one longer code): false once the parse has ended (at
// `stop`, or invalid).
__device__ __forceinline__ bool sync_step(WinReader& r, uint32_t stop, uint32_t limit, uint32_t& n, bool& invalid) {
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

// The parse passes' chunk interiors: a branchless step (round 4).  The interior loops of round 3 branched
// per step (refill, run marks, long code, code mark); every branch is exec-mask bookkeeping on the scalar
// unit and a wave ran each branch any of its lanes took.  Measured (c8, one box, A/B x 2): sync 625 ->
// 558 us, mark 896 -> 798 us.  Two chunks per thread interleaved through the same step ran slower (739 /
// 961 us: half the waves, and the compiler did not interleave the chains), not kept.
// WinReader's state inside a chunk's interior as 32-bit words: bits [pos, pos + avail) left-aligned in
// hi:lo and zero past avail, the word after them (index nx) in pre; pos = 32 nx - avail.
struct Lean {
    uint32_t hi, lo, avail, nx, pre;
    __device__ __forceinline__ uint32_t pos() const { return nx * 32u - avail; }
};
__device__ __forceinline__ Lean lean_from(const WinReader& r) {
    return Lean{(uint32_t)(r.buf >> 32), (uint32_t)r.buf, (uint32_t)r.avail, r.next, r.pre};
}
__device__ __forceinline__ void lean_to(WinReader& r, const Lean& c) {
    r.buf = ((uint64_t)c.hi << 32) | c.lo;
    r.avail = (int)c.avail;
    r.next = c.nx;
    r.pos = c.pos();
    r.pre = r.s[c.nx < r.n ? c.nx : 0u];
}

// The window word reader of the lean steps (a functor: the interior loops were measured with other window
// layouts)
struct WinRead {
    const uint32_t* s;
    __device__ __forceinline__ uint32_t operator()(uint32_t i) const { return s[i]; }
};

// One branchless step inside the interior (every word read lies in the window): a run of 1-bit codes
// (value 0) of up to 31 -- a run never extends past avail, whose bits are zero -- then a refill to >= 32
// bits, then the longer code that follows the run if there is one.  Returns the values taken (<= 32);
// bad: that code has >= 33 bits or 32 leading zeros (left unconsumed for the checked loop).  A run cut
// short by avail takes no code; the next step continues it.  BOUNDED: room (>= 1) bits are left before
// the parse's stop; the run ends there at the latest and a code is taken only if it starts before it,
// so the parse ends exactly at the first code boundary at or past the stop (the code may reach past).
// CAP: the run's cap when unbounded (31).  n1_out / w_out: the run's length and the code's width (0: none).
template <bool BOUNDED = false, uint32_t CAP = 31u, class Rd>
__device__ __forceinline__ uint32_t lean_step(const Rd& s, Lean& c, bool& bad, uint32_t room = 32u,
                                              uint32_t* n1_out = nullptr, uint32_t* w_out = nullptr) {
    // ones at the top of hi, at most CAP (BOUNDED: at most room): the OR-ed bit makes clz defined and caps it
    const uint32_t cap_bit = BOUNDED ? 0x80000000u >> min(room, 31u) : 0x80000000u >> CAP;
    uint32_t n1 = __builtin_clz(~c.hi | cap_bit);
    uint64_t b = (((uint64_t)c.hi << 32) | c.lo) << n1;
    c.avail -= n1;
    // a 0 bit follows the run: a code starts (BOUNDED: before the stop)
    const bool has = c.avail != 0u && (uint32_t)(b >> 63) == 0u && (!BOUNDED || n1 < room);
    uint32_t hi = (uint32_t)(b >> 32), lo = (uint32_t)b;
    // refill: append pre when fewer than 32 bits are buffered (branchless; the re-read of pre is
    // unconditional, the same word when nothing was appended)
    const bool need = c.avail < 32u;
    const uint32_t rh = hi | (c.pre >> (c.avail & 31u));
    const uint32_t rl = __builtin_amdgcn_alignbit(c.pre, 0u, c.avail);  // pre << (32 - avail); 0 at avail 0
    hi = need ? rh : hi;
    lo = need ? rl : lo;
    c.avail += need ? 32u : 0u;
    c.nx += need ? 1u : 0u;
    c.pre = s(c.nx);
    const uint32_t zz = hi ? (uint32_t)__builtin_clz(hi) : 32u;
    bad = has && zz >= 16u;
    const bool take = has && zz < 16u;
    const uint32_t w = take ? 2u * zz + 1u : 0u;
    b = (((uint64_t)hi << 32) | lo) << w;
    c.hi = (uint32_t)(b >> 32);
    c.lo = (uint32_t)b;
    c.avail -= w;
    if (n1_out) *n1_out = n1;
    if (w_out) *w_out = w;
    return n1 + (take ? 1u : 0u);
}
// The interior loops run while the parse is a margin short of every bound.  A step's reads past the bound
// stay inside the block window (the last chunk's bound has the 256-bit slack behind it), so only the bits
// a step takes must stay short of it: the table steps of both passes take <= 31 + 31 bits; the bounded
// steps then finish the chunk.  (128, the window-read bound, before: sync 346 -> 311 us, mark 464 -> 442
// us per c8 step with its former two-code step, A/B x 3 on one box, profiles/r05/c8_ab.)
constexpr uint32_t kLeanMargin = 64;
static_assert(31 + 31 < kLeanMargin && 31 * 8 < 256, "steps stay short of the bound");

// Sync-pass step by table (round 5): a run of 1-bit codes as lean_step, a refill to >= 32 bits, then every
// code that lies wholly in the next kEgLutBits bits at once, from a 4 KiB table of (codes, bits) per bit
// pattern; no code complete in them (a code of more than kEgLutBits bits): one code by its leading zeros.
// A step moves at most 31 + 31 bits (kLeanMargin).  The sync pass needs only the count and the exit, so the
// codes' individual boundaries are never formed.
// Table width of the mark pass (12: 4 KiB, 5 blocks per CU beside its window and mark slots) and of the
// sync pass (DCT3D_SYNC_LUT_BITS, default 12: 7 blocks per CU)
constexpr int kEgLutBits = 12;
#ifndef DCT3D_SYNC_LUT_BITS
#define DCT3D_SYNC_LUT_BITS 12
#endif
constexpr int kSyncLutBits = DCT3D_SYNC_LUT_BITS;
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
__device__ constexpr EgLut<kEgLutBits> kEgLut = make_eg_lut<kEgLutBits>();
__device__ constexpr EgLut<kSyncLutBits> kSyncLut = make_eg_lut<kSyncLutBits>();
// the block's copy of a table: 16-byte pieces, ordered by the staging's barrier
template <int B>
__device__ __forceinline__ void copy_lut(uint8_t* s_lut, const EgLut<B>& t) {
    static_assert((1 << B) % (16 * kEgBlock) == 0, "whole 16-byte pieces per thread");
#pragma unroll
    for (int r = 0; r < (1 << B) / (16 * kEgBlock); r++)
        *(uint4*)(s_lut + 16 * (threadIdx.x + r * kEgBlock)) = *(const uint4*)(t.e + 16 * (threadIdx.x + r * kEgBlock));
}
static_assert(kEgLutBits <= 15 && kSyncLutBits <= 15, "counts and widths fit 4 bits");

template <int B, class Rd>
__device__ __forceinline__ uint32_t lean_step_lut(const Rd& s, const uint8_t* lut, Lean& c, bool& bad) {
    const uint32_t n1 = __builtin_clz(~c.hi | 1u);  // run of 1-bit codes, at most 31, never past avail
    uint64_t b = (((uint64_t)c.hi << 32) | c.lo) << n1;
    c.avail -= n1;
    uint32_t hi = (uint32_t)(b >> 32), lo = (uint32_t)b;
    const bool need = c.avail < 32u;  // refill (as lean_step): the run ended on a code boundary either way
    const uint32_t rh = hi | (c.pre >> (c.avail & 31u));
    const uint32_t rl = __builtin_amdgcn_alignbit(c.pre, 0u, c.avail);
    hi = need ? rh : hi;
    lo = need ? rl : lo;
    c.avail += need ? 32u : 0u;
    c.nx += need ? 1u : 0u;
    c.pre = s(c.nx);
    const uint32_t e = lut[hi >> (32 - B)];
    const uint32_t k = e & 15u;
    const uint32_t zz = hi ? (uint32_t)__builtin_clz(hi) : 32u;
    const bool one = k == 0u && zz < 16u;  // one code of 13 .. 31 bits
    bad = k == 0u && zz >= 16u;            // >= 33 bits or invalid: the checked loop reads it
    const uint32_t w = k ? e >> 4 : (one ? 2u * zz + 1u : 0u);
    b = (((uint64_t)hi << 32) | lo) << w;
    c.hi = (uint32_t)(b >> 32);
    c.lo = (uint32_t)b;
    c.avail -= w;
    return n1 + (k ? k : (one ? 1u : 0u));
}

// The mark pass's table step: lean_step_lut that stops on the step's one possible mark.  d0: the values
// before the next mark.  All k table codes are taken unless the step's values would pass 32 (two marks) or
// the mark falls on the table's second .. k-th code, whose bit offsets the table does not give; then only
// the first code (its width by clz).  The mark is then always the run's d0-th value or the first code: bit
// p0 + d0 of the step.  A step moves at most 31 + 31 bits.  (Round 5: the two-code step before it -- a run
// of <= 30, a code, a second code when buffered, 53 VALU with the mark -- against 46 VALU and 9 % / 25 %
// fewer steps on ramp / uniform content: the pass 430 -> 356 us per c8 step although its 4 KiB table costs
// a sixth block per CU, profiles/r05/mark_lut.)
template <class Rd>
__device__ __forceinline__ uint32_t lean_step_lut_mark(const Rd& s, const uint8_t* lut, Lean& c, bool& bad,
                                                       uint32_t d0) {
    const uint32_t n1 = __builtin_clz(~c.hi | 1u);
    uint64_t b = (((uint64_t)c.hi << 32) | c.lo) << n1;
    c.avail -= n1;
    uint32_t hi = (uint32_t)(b >> 32), lo = (uint32_t)b;
    const bool need = c.avail < 32u;
    const uint32_t rh = hi | (c.pre >> (c.avail & 31u));
    const uint32_t rl = __builtin_amdgcn_alignbit(c.pre, 0u, c.avail);
    hi = need ? rh : hi;
    lo = need ? rl : lo;
    c.avail += need ? 32u : 0u;
    c.nx += need ? 1u : 0u;
    c.pre = s(c.nx);
    const uint32_t e = lut[hi >> (32 - kEgLutBits)];
    const uint32_t k = e & 15u;
    const uint32_t zz = hi ? (uint32_t)__builtin_clz(hi) : 32u;
    const bool full = k != 0u && n1 + k <= 32u && d0 - n1 - 1u >= k - 1u;
    const bool one = !full && zz < 16u;
    bad = !full && zz >= 16u;
    const uint32_t w = full ? e >> 4 : (one ? 2u * zz + 1u : 0u);
    b = (((uint64_t)hi << 32) | lo) << w;
    c.hi = (uint32_t)(b >> 32);
    c.lo = (uint32_t)b;
    c.avail -= w;
    return n1 + (full ? k : (one ? 1u : 0u));
}

// The resolve walk of chunk t (pass 0 with resolve, below): e = the pass-0 exit of chunk t - 1 (~0u: it
// ended invalid), s0 = chunk t's pass-0 start, x0 = its pass-0 exit (window-relative), n = its pass-0
// count, ex = its pass-0 exit (absolute).  On return n / exit are chunk t's true count and exit; true
// (fail) when the true exit differs from the pass-0 exit that chunk t + 1 was resolved against.
__device__ __forceinline__ bool resolve_chunk(const uint32_t* win, uint32_t e, uint32_t s0, uint32_t x0, uint32_t stop,
                                              uint32_t limit, uint64_t base, uint64_t ex, uint32_t& n, uint64_t& exit) {
    if (e == ~0u) return false;
    bool met = false;
    if (e - s0 < kMeetBits) {  // e >= s0: the exit of chunk t - 1 lies at or past its end
        WinReader a{win, kSyncWinWords, 0, 0, 0, 0, 0};  // pass 0, from s0
        WinReader q{win, kSyncWinWords, 0, 0, 0, 0, 0};  // the true parse, from e
        a.seek(s0);
        q.seek(e);
        uint32_t na = 0, nq = 0, code;
        for (;;) {
            if (a.pos == q.pos) {  // met: a boundary of both parses
                met = a.pos <= x0;  // ... at or before the pass-0 exit (else: past the data's end)
                if (met) n = n - na + nq;
                break;
            }
            if (min(a.pos, q.pos) - s0 >= kMeetBits || max(a.pos, q.pos) > limit) break;
            const bool adv_a = a.pos < q.pos;  // the one behind takes its next code
            if (!(adv_a ? a.get(code) : q.get(code))) break;  // 32 zero bits
            if (adv_a) na++;
            else nq++;
        }
    }
    if (met) return false;
    // rare (a dense run of long codes): the confirming pass of this chunk, inline
    WinReader q{win, kSyncWinWords, 0, 0, 0, 0, 0};
    q.seek(e);
    uint32_t n2 = 0;
    bool inv2 = false;
    while (q.pos < stop && sync_step(q, stop, limit, n2, inv2)) {
    }
    n = n2;
    exit = inv2 ? kNoExit : base + q.pos;
    // chunk t + 1 was resolved against the pass-0 exit: only a different true exit needs the confirming
    // passes
    return exit != ex;
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
// is status[0] set, and the host then runs confirming passes (iteration 1, plain mapping).
__global__ __launch_bounds__(kEgBlock) void eg_sync_kernel(EgDecParams P, int iteration, int resolve) {
    __shared__ uint32_t win[kSyncWinAlloc];
    __shared__ uint32_t s_exit[kEgBlock];
    __shared__ __attribute__((aligned(16))) uint8_t s_lut[1 << kSyncLutBits];
    copy_lut(s_lut, kSyncLut);
    const bool rs = iteration == 0 && resolve;
    const uint64_t b = blockIdx.x;
    const uint64_t first = rs ? (b ? b * (kEgBlock - 1) - 1 : 0) : b * kEgBlock;
    const LdsBits L = stage_block_window(P, win, first);
    // rs: block 0's thread 0 has no helper chunk (t = -1 wraps: past n_chunks)
    const uint64_t t = rs ? b * (kEgBlock - 1) + threadIdx.x - 1 : first + threadIdx.x;
    const bool live = t < P.n_chunks;
    const uint64_t base = L.w0 * 32;
    const uint32_t end = rel_bit(P.start_bit + (t + 1) * kChunkBits, base);
    const uint32_t limit = rel_bit(P.limit_bit, base);
    const uint32_t stop = min(end, limit);
    WinReader r{win, kSyncWinWords, 0, 0, 0, 0, 0};
    const uint32_t s0 = live ? rel_bit(chunk_start(P, t, iteration), base) : 0u;
    uint32_t n = 0;
    bool invalid = false;
    if (live) {
        r.seek(s0);
        // exactly the codes a one-at-a-time parse reads: every 1-bit code boundary is a code boundary.
        // The chunk interior first, without bounds (kLeanMargin; by table: lean_step_lut), then the bounded
        // steps to the chunk end, then the checked steps; a long or invalid code leaves the lean loops
        // unconsumed.
        const uint32_t fast_stop = stop > kLeanMargin ? stop - kLeanMargin : 0u;
        // the bounded steps end the parse exactly at the stop -- unless the data ends within reach of the
        // chunk end (a code running past the limit is invalid: the checked steps)
        const uint32_t bstop = limit >= stop + 64u ? stop : 0u;
        Lean c = lean_from(r);
        bool bad = false;
        const WinRead rd{win};
        while (!bad & (c.pos() < fast_stop)) n += lean_step_lut<kSyncLutBits>(rd, s_lut, c, bad);
        while (!bad & (c.pos() < bstop)) n += lean_step<true>(rd, c, bad, bstop - c.pos());
        lean_to(r, c);
        while (r.pos < stop && sync_step(r, stop, limit, n, invalid)) {
        }
    }
    const uint64_t ex = invalid ? kNoExit : base + r.pos;
    if (!rs) {
        if (!live) return;
        P.exit_out[t] = ex;
        P.count[t] = n;
        if (iteration > 0 && ex != P.exit_in[t]) atomicOr((unsigned int*)&P.status[0], 1u);
        return;
    }
    s_exit[threadIdx.x] = invalid ? ~0u : r.pos;
    __syncthreads();
    if (!live || threadIdx.x == 0) return;  // thread 0: the helper chunk (written by its owner block)
    uint64_t exit = ex;
    const bool fail = t > 0 && resolve_chunk(win, s_exit[threadIdx.x - 1], s0, r.pos, stop, limit, base, ex, n, exit);
    P.exit_out[t] = exit;
    P.count[t] = n;
    const uint64_t fb = __ballot(fail);
    if (fb != 0ull && (threadIdx.x & 63) == (uint32_t)__builtin_ctzll(fb)) atomicOr((unsigned int*)&P.status[0], 1u);
}

// The chunk's marks are collected in LDS (2 bytes each, relative to the chunk's true start, in the
// thread's own slot of kMkSlot entries) and written out at the end, each thread its consecutive marks back
// to back, so that the L2 assembles whole lines: WRITE_SIZE 1.67 GB -> 0.52 GB (the marks' own bytes) and
// the pass 708 -> 529 us on one box (round 4; stored one at a time as the parse reached them, through a
// buffer descriptor, each lane's marks tens of microseconds apart, the lines were written back partial).
// The slots cost 8.5 KiB per block (with the window, 6 blocks per CU instead of 8).  A step's one possible
// mark is stored branch-free: steps without a mark store to the thread's dummy, 2 bytes behind the
// window (round 4: an 18th slot entry; an exec-masked store instead compiled to a branch and 13 more VALU
// per step).
// Marks leave as the low 16 bits of their bit position (round 5; 64-bit before: 0.52 GB written and read
// back per c8 step, then 32-bit: 0.27 GB), the whole position of every 64th (a consumer group's first) in
// mark_base (mark_offset).
constexpr uint32_t kMkSlot = 17;  // a chunk has at most 17 marks (<= 512 values)
__global__ __launch_bounds__(kEgBlock) void eg_mark_kernel(EgDecParams P) {
    __shared__ uint32_t win[kSyncWinAlloc];
    __shared__ uint16_t s_mk[kEgBlock * kMkSlot];
    __shared__ __attribute__((aligned(16))) uint8_t s_lut[1 << kEgLutBits];
    copy_lut(s_lut, kEgLut);
    // the sync pass's verdict: status[0] != 0 only after a speculative pass 0 whose chunks did not all
    // resolve (the converged confirming passes leave it 0): no marks, the consumers skip themselves
    // (status[2] != 0) and the host reruns without speculation
    if (P.status[0] != 0) {  // grid-uniform
        if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr((unsigned int*)&P.status[2], 4u);
        return;
    }
    const uint64_t first = (uint64_t)blockIdx.x * kEgBlock;
    // (the per-chunk loads below issued before the window's staging instead measured 633 -> 745 us)
    const LdsBits L = stage_block_window(P, win);
    const uint64_t t = first + threadIdx.x;
    if (t >= P.n_chunks) return;
    // the chunk's first value index and true start: both loads in flight together, at the top issue
    // priority (one round trip, not two behind the other blocks' parse work)
    __builtin_amdgcn_s_setprio(3);
    const uint64_t idx0 = P.off[t];
    // the converged exits are in exit_in (the host swaps the buffers after every pass)
    const uint64_t s = t == 0 ? P.start_bit : P.exit_in[t - 1];
    __builtin_amdgcn_s_setprio(0);
    if (idx0 >= P.n_values) return;
    if (s == kNoExit) return;  // the true parse stopped in an earlier chunk: reported by that chunk
    const uint64_t base = L.w0 * 32;
    const uint32_t end = rel_bit(P.start_bit + (t + 1) * kChunkBits, base);
    const uint32_t limit = rel_bit(P.limit_bit, base);
    WinReader r{win, kSyncWinWords, 0, 0, 0, 0, 0};
    const uint32_t sp = rel_bit(s, base);  // the chunk's true start (LDSM marks are relative to it)
    r.seek(sp);
    uint16_t* const myk = s_mk + threadIdx.x * kMkSlot;  // mark k of the chunk (value 32 k - ph) at myk[k]
    uint16_t* const dummy = (uint16_t*)(win + kSyncWinWords) + threadIdx.x;  // a step without a mark stores here
    // chunk-relative 32-bit value count i (value idx0 + i): the 64-bit index arithmetic per step was a
    // large part of the pass.  A chunk holds at most ~kChunkBits + 64 codes, so rem below never binds
    // unless the wanted values end inside this chunk.
    const uint64_t rem64 = P.n_values - idx0;
    const uint32_t rem = (uint32_t)min(rem64, (uint64_t)(2 * kChunkBits));
    const bool ends_here = rem64 <= 2 * kChunkBits;
    const uint32_t ph = (uint32_t)idx0 & (kMarkVals - 1);
    const uint64_t gm0 = idx0 / kMarkVals;  // mark gm0 + k = mark of value idx0 + 32 k - ph
    uint32_t i = 0, code;
    // Interior of the chunk: a step moves at most 31 + 31 bits and 32 values, so while the parse is
    // kLeanMargin bits short of the chunk end and of the data limit none of the bounds below can bind -- a
    // lean loop without them (a long or invalid code leaves it for the checked loop, which reads or reports
    // it).  The lean loops run only in chunks that cannot hold the last wanted value (rem64 > 2 kChunkBits;
    // the few others take the checked steps whole): there the value count never binds, and the loops test
    // only the position (round 5: 53 -> 50 VALU per step with the running mark index and slot below).
    const uint32_t lim_end = ends_here ? 0u : min(end, limit);
    const uint32_t fast_end = lim_end > kLeanMargin ? lim_end - kLeanMargin : 0u;
    {
        Lean c = lean_from(r);
        bool bad = false;
        const WinRead rd{win};
        // the next mark: chunk-relative value index nm (value idx0 + nm), its slot mp; a step takes nv <= 32
        // values, so at most one mark, value d0 = nm - i of the step
        uint32_t nm = (0u - ph) & (kMarkVals - 1);
        uint16_t* mp = myk + (ph + nm) / kMarkVals;
        const uint32_t s0 = 0u - sp;  // (bit positions leave relative to the chunk's true start)
        auto mark = [&](uint32_t at, uint32_t nv, uint32_t d0) {
            const bool hit = d0 < nv;
            *(hit ? mp : dummy) = (uint16_t)(at + s0);  // no branch
            nm += hit ? kMarkVals : 0u;
            mp += hit ? 1 : 0;
            i += nv;
        };
        // table steps that stop on the mark (nv <= 32): the mark is value d0 of the step, at bit p0 + d0
        while (!bad & (c.pos() < fast_end)) {
            const uint32_t p0 = c.pos();
            const uint32_t d0 = nm - i;
            mark(p0 + d0, lean_step_lut_mark(rd, s_lut, c, bad, d0), d0);
        }
        // to the chunk end exactly (as the sync pass; the chunk holding the last wanted value and the data's
        // end take the checked steps)
        const uint32_t bend = limit >= end + 64u && !ends_here ? end : 0u;
        while (!bad & (c.pos() < bend)) {
            const uint32_t p0 = c.pos();
            const uint32_t d0 = nm - i;
            mark(p0 + d0, lean_step<true>(rd, c, bad, bend - p0), d0);
        }
        lean_to(r, c);
    }
    while (i < rem && r.pos < end) {
        const uint32_t p0 = r.pos;
        if (p0 >= limit) {  // ran out of bits
            atomicOr((unsigned int*)&P.status[2], 2u);
            return;
        }
        // one step = a run of 1-bit codes, then one longer code (as sync_step): every lane advances
        // through both halves each iteration, instead of the wave running a run-only and a code-only
        // iteration for lanes that are in different halves
        const uint32_t room = min(min(end - p0, limit - p0), rem - i);
        const uint32_t k = r.ones(min(room, 64u));
        if (k) {  // values i .. i + k - 1 are zeros at bits p0 .. p0 + k - 1
            for (uint32_t j = ((ph + i + kMarkVals - 1) & ~(kMarkVals - 1)) - ph; j < i + k; j += kMarkVals)
                myk[(ph + j) / kMarkVals] = (uint16_t)(p0 + (j - i) - sp);
            i += k;
            if (ends_here && i == rem) P.status[1] = base + r.pos;  // the bit after the last wanted value
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
        if (((ph + i) & (kMarkVals - 1)) == 0) myk[(ph + i) / kMarkVals] = (uint16_t)(p1 - sp);
        if (++i == rem && ends_here) P.status[1] = base + r.pos;
    }
    // the chunk's marks k = (ph ? 1 : 0) .. (ph + i - 1) / 32, back to back
    const uint64_t b0 = base + sp;
    uint16_t* const mk = P.mark + gm0;
    for (uint32_t k = ph ? 1u : 0u; k < (ph + i + kMarkVals - 1) / kMarkVals; k++) {
        const uint64_t m = b0 + myk[k];
        mk[k] = (uint16_t)m;
        if (((gm0 + k) & (kMarkGroup - 1)) == 0) P.mark_base[(gm0 + k) / kMarkGroup] = m;
    }
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

int launch_eg_mark(const EgDecParams& P, hipStream_t st) {
    if (P.n_chunks == 0) return 0;
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
