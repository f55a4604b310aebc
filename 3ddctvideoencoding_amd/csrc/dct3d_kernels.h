// dct3d_kernels.h -- kernel parameter blocks and launchers (shared by dct3d_kernels.hip and the
// C-ABI runtime dct3d_runtime.cpp).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace dct3d {

constexpr int kMaxGroupsDev = 64;  // == kMaxGroups in dct3d_plan.h; one LDS slot per lane
constexpr int kGM4Dev = 48;        // == kMaxGroups4 in dct3d_plan.h (8x8x4 in-wave fold, per cube)
// Per-call counters of the in-wave paths are spread over kCountSpread words per counter (a block adds
// to word blockIdx & (kCountSpread - 1)): 10^5 same-address atomics per call serialise at the L2
// (~12 ns each, longer than the whole kernel); the host sums the words.
constexpr int kCountSpread = 512;

// n / d for n < 2^31 as one 32x32->64 multiply and a shift (Granlund-Montgomery: s = 31 + ceil(log2 d),
// m = ceil(2^s / d) < 2^32 gives floor(n m / 2^s) = floor(n / d) for every n < 2^31); set_fast_div
// (dct3d_runtime.cpp) fills m and s on the host
struct FastDiv {
    uint32_t m, s;
};

struct EncodeParams {
    const uint8_t* raster;
    int32_t* out;
    uint32_t n_cubes;          // end of this launch's cube range (global index, whole stacks)
    uint32_t g_base;           // first cube of this launch (global index; 0 unless a tail launch)
    uint32_t cubes_per_stack;
    uint32_t nbx;              // cubes per block-row
    FastDiv div_cps, div_nbx;  // the two divisions of the cube -> raster address map
    uint32_t width;
    uint64_t plane;            // width * height
    uint64_t stack_stride;     // D * plane
    double coef_dc;            // Java DC group coefficient
    const float* tab_rstep;    // [32] fp32(1/step_s)
    const float* tab_G;        // [32]
    const float* tab_E;        // [32]
    // uncertified coefficients are replayed inside the wave (exact Java fold, DCT.java:44-52)
    const int32_t* ngroups;    // [cs] fold length of each coefficient
    const double* coef;        // [cs * kMaxGroupsDev]
    const uint8_t* group_of;   // [cs * cs]
    unsigned int* replay_count;  // this call's counter slot: [0, S) Java-fold replays, [S, 2S) fp64
                                 // settlements (S = kCountSpread words each), or nullptr
    unsigned int* replay_clear;  // the other slot (2S words): zeroed by block 0 for the next call
    const double* tab64;       // 8x8x8 second certificate: [64] fp64 basis [k][n], [32] thresholds per s
    uint32_t recheck;          // 1: run the second certificate (0: test option, all open -> Java fold)
    uint64_t* trace;           // MODE 3 (diagnostic timeline): per wave {start, transform done, stored, hw id}
    // MODES 4 / 5 (diagnostic traversal sweep): the waves walk the cubes in vertical strips of strip_w
    // cubes (strip_cubes = strip_w * block rows per stack), row-major within a strip (strip_cube)
    uint32_t strip_w, strip_cubes;
    FastDiv div_strip_w, div_strip_cubes;
};

struct DecodeParams {
    const int32_t* in;
    uint8_t* out;
    uint32_t n_cubes, cubes_per_stack, nbx, width;
    FastDiv div_cps, div_nbx;
    uint32_t cube_base;        // decode_eg_kernel: first cube of this launch (a chunk of whole stacks)
    uint64_t plane, stack_stride;
    double dec_G, dec_E;       // certificate: margin = dec_G * sum |dequantised| + dec_E
    float dec_l1_max;          // sum |dequantised| >= this: the cube goes to the exact replay
    uint32_t blk_store;        // 1: full blocks store whole lines through LDS (nbx even, a stack < 4 GiB)
    // uncertified cubes are replayed whole inside the wave (exact Java InverseDCT fold)
    const double* inv_coef_t;    // [cs * cs], transposed: inv_coef_t[k * cs + n] = coefficients[n][k]
    unsigned int* replay_count;  // this call's counter slot: [0, S) cubes replayed (S = kCountSpread), or nullptr
    unsigned int* replay_clear;  // the other slot (2S words): zeroed by block 0 for the next call
};

struct Fwd64Params {
    const uint8_t* raster;
    double* out;
    uint32_t n_cubes, cubes_per_stack, nbx, width;
    uint64_t plane, stack_stride;
};

int launch_cube_f32(int D, bool inverse, const float* in, float* out, uint32_t n_cubes, hipStream_t st);
int launch_fwd64_raster(int D, const Fwd64Params& P, hipStream_t st);
int launch_encode(int D, const EncodeParams& P, hipStream_t st);
struct EgParams {
    const int32_t* q;          // cube-major quantised values
    uint64_t n_cubes;
    const uint16_t* diag;      // [cs] diagonal-slice order: cube index x + 8y + 64z per stream position
    uint32_t* bits;            // [n_cubes] bits per cube
    uint64_t* off;             // [n_cubes] stream bit offset of each cube (carry included)
    uint64_t* bsum;            // [n_chunks] chunk sums -> chunk offsets
    uint64_t* status;          // [0] total bits (carry included), [1] flags: 1 capacity, 2 value range
    uint32_t* head;            // [n_cubes] first output word of each cube (memory byte order)
    uint32_t* tail;            // [n_cubes] last output word of each cube
    uint32_t* out;             // output words (memory byte order), capacity out_cap_words
    uint64_t out_cap_words;
    uint32_t carry_bits, carry_byte;
    // (eg_stitch_kernel, optional) the host's pinned copy of status[0..1], written by block 0, and the other
    // of the ctx's two status slots, zeroed for the next call (no copy kernel and no memset per call)
    uint64_t* status_host;
    uint64_t* status_clear;
    uint64_t seq;  // (with status_host) the call's tag: [7] = hand_off_tag(seq, total bits, flags), polled by the host
};

// A call's verdict as one 64-bit word (hand-off to the host while the call's last kernels still run): the
// call's sequence number (low 16 bits) in bits 63..48, flags in 47..40, a value < 2^40 in 39..0 (flag 0x80:
// the value did not fit -- the host then waits for the stream and reads the whole words).  One store, so
// the host never sees part of it, and no ordering against other stores is needed: the device writes it
// with a system-scope relaxed store (written through; a release would write back the whole L2 first,
// measured no faster).
constexpr uint64_t kTagValueMask = (1ull << 40) - 1;
constexpr uint32_t kTagOverflow = 0x80;
__host__ __device__ inline uint64_t hand_off_tag(uint64_t seq, uint64_t value, uint32_t flags) {
    if (value > kTagValueMask) flags |= kTagOverflow;
    return ((seq & 0xFFFFull) << 48) | ((uint64_t)(flags & 0xFF) << 40) | (value & kTagValueMask);
}

// Exp-Golomb decode (self-synchronising chunks, see dct3d_eg.hip)
constexpr uint64_t kEgChunkBits = 512;  // bits per parse chunk (one thread each)
// Marks (the bit position of every 32nd value) are stored as their low 16 bits; the whole position of a
// group's first (kMarkGroup marks: a consumer wave's 2,048 values) is kept in mark_base.  Consecutive
// marks lie < 2^16 bits apart (32 codes of < 64 bits), so a mark's offset from its group's first is the
// sum of the 16-bit differences up to it: a wave holding the group's 64 marks counts the wraps
// (mark_offset), a single lane adds the differences (mark_serial).  (Round 5: 32-bit low halves before,
// 0.27 GB written by the mark pass and read back by the consumer per c8 step.)
constexpr uint64_t kMarkGroup = 64;
struct EgDecParams {
    const uint32_t* words;     // stream, memory byte order
    uint64_t n_words;
    uint64_t start_bit, limit_bit;  // first bit of the stream, end of the available bits
    uint64_t n_chunks;
    uint64_t n_values;         // values wanted (n_cubes * cs)
    int cs;
    const uint16_t* diag;
    uint64_t* exit_in;         // previous iteration's exits (UINT64_MAX: the parse ended invalid)
    uint64_t* exit_out;
    uint32_t* count;           // codewords per chunk
    uint64_t* off;             // (unused by the stream decode since round 6: the mark pass scans its block)
    // the scan of the counts (launch_eg_dscan): bsum[b] = the value index of chunk 4096 b's first codeword,
    // part[i] = the codewords of chunks 256 i .. 256 i + 255
    uint64_t* bsum;
    uint32_t* part;
    // [0] changed / first invalid chunk, [1] end bit, [2] flags (1 corrupt, 2 short, 4 rerun), [3] a code of
    // 33+ bits seen (mark pass; the consumers then parse with CHECK); zeroed with the other words by
    // eg_decode_front's memset before every pass
    uint64_t* status;
    uint16_t* mark;            // [n_values / 32] bit position of every 32nd value, low 16 bits
    uint64_t* mark_base;       // [n_values / 32 / kMarkGroup + 1] bit position of every kMarkGroup-th mark
    int32_t* q;                // cube-major output
    // (decode_eg_kernel, optional) the host's pinned copy of status[0..5], written by block 0 as it starts
    // (every word is final by then), and [6] = hand_off_tag(seq, end bit, verdict flags): the host polls
    // for it and returns while the consumer still runs (the raster completes on the stream, as every *_dev
    // output)
    uint64_t* status_host;
    uint64_t seq;
    // (decode_eg_kernel, optional) the ctx's other status slot, zeroed by block 0 for the next call (whose
    // front then needs no memset)
    uint64_t* status_clear;
};

// Fused encode + Exp-Golomb (dct3d_encode_eg_dev): the encode kernel's transform / quantise /
// certify, the exact Java replay of uncertified coefficients inside the wave, then the wave's 8
// cubes coded straight into a private slot (no int32 cube-major round trip).  Segment = one wave = 8
// consecutive cubes; lane l codes 1/8 of one cube's diagonal stream at its bit offset in the segment.

struct EgFusedParams {
    const int32_t* ngroups;    // exact replay tables (as EncodeParams)
    const double* coef;
    const uint8_t* group_of;
    const uint16_t* diag;      // [cs] stream position -> cube index
    uint32_t* slot;            // [n_seg * seg_cap]: the segment's stream, MSB-first words, its first bit
                               // at bit 31 of word 0
    uint32_t seg_cap;          // 64 * words per lane (worst case cs/8 values x 27 bits)
    uint32_t* seg_bits;        // [n_seg] bits per segment (the scan's input)
};

// Lane l of a wave holding a group's marks in order (lane 0: the group's first, base_low its low 16 bits;
// lanes past the last mark: any value) -> the offset of its mark from the group's first: the 16-bit
// difference r_l plus 2^16 per wrap at or below l (a wrap: r_l < r_{l-1}).  All 64 lanes take part.
__device__ __forceinline__ uint32_t mark_offset(uint32_t low, uint32_t base_low) {
    const uint32_t r = (low - base_low) & 0xFFFFu;
    const uint32_t prev = __shfl_up(r, 1);  // lane 0: its own (0)
    const bool wrap = r < prev;
    const uint64_t wraps = __ballot(wrap);
    const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(wraps >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)wraps, 0u));
    return r + ((below + (uint32_t)wrap) << 16);
}
// the whole bit position of mark m, one lane alone (the exact replay): the differences from its group's first
__device__ __forceinline__ uint64_t mark_serial(const uint16_t* mark, const uint64_t* mark_base, uint64_t m) {
    const uint64_t g0 = m & ~(kMarkGroup - 1), gb = mark_base[m / kMarkGroup];
    uint32_t off = 0, prev = (uint16_t)gb;
    for (uint64_t k = g0 + 1; k <= m; k++) {
        const uint32_t c = mark[k];
        off += (c - prev) & 0xFFFFu;
        prev = c;
    }
    return gb + off;
}

int launch_decode(int D, const DecodeParams& P, hipStream_t st);
int launch_encode_eg(int D, const EncodeParams& P, const EgFusedParams& E, hipStream_t st);
int launch_eg_stitch(const EgParams& P, hipStream_t st);
// scan of the segment bits + the lanes' words concatenated into the stream + stitch (P.n_cubes =
// segments, P.bits = seg_bits)
int launch_eg_compact(const EgParams& P, const uint32_t* slot, uint32_t seg_cap, hipStream_t st);
int launch_eg_encode(int D, const EgParams& P, hipStream_t st);
// resolve (pass 0): each chunk's true parse is followed from the exit of chunk t - 1 until it meets a
// pass-0 boundary of chunk t (in the block's LDS window); status[0] = 0: every chunk met, the pass-0 exits
// and counts are final.  Otherwise (or without resolve) confirming passes (iteration 1) follow.
int launch_eg_sync(const EgDecParams& P, int iteration, int resolve, hipStream_t st);
int launch_eg_scan(const EgParams& P, hipStream_t st);   // scan of P.bits[0..n_cubes) into P.off / P.status[0]
int launch_eg_decode_write(int D, const EgDecParams& P, hipStream_t st);  // mark pass + emit
int launch_eg_mark(const EgDecParams& P, hipStream_t st);
// the stream decode's scan of the chunk counts: P.bsum (exclusive, per 4,096 chunks), P.part (per 256) and
// the total (S.status[0]); S: the scan's status words and the generic scan's parameters
int launch_eg_dscan(const EgDecParams& P, const EgParams& S, hipStream_t st);
// the fused front (resolving sync pass + scan + mark pass in one launch; desc: front_blocks(n_chunks) zeroed
// words); a chunk that does not resolve: status[2] bit 4 (rerun without speculation)
uint64_t front_blocks(uint64_t n_chunks);
int launch_eg_front(const EgDecParams& P, uint64_t* desc, int force_fail, hipStream_t st);
int launch_eg_emit(int D, const EgDecParams& P, hipStream_t st);
// fused stream -> raster decode: values parsed at the marks straight into the decode's LDS staging
// groups_per_wave: 1, 2, 4 or 8 (other values: 8) groups of CPW cubes per wave, the next one's loads ahead
int launch_decode_eg(int D, const DecodeParams& P, const EgDecParams& E, int groups_per_wave, hipStream_t st);

}  // namespace dct3d
