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
//   eg_zero_kernel    clears the output words and seeds word 0 with the carried partial byte
//   eg_write_kernel   one wave per cube: lane-level exclusive scan of code lengths, codes OR-ed into
//                     a wave-private LDS image aligned to the cube's first output word, stored as
//                     stream-order words (byte-swapped); the two words a cube may share with its
//                     neighbours are merged with atomicOr, the interior words are plain stores.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "dct3d_kernels.h"

namespace dct3d {
namespace {

constexpr int kEgBlock = 256;
constexpr int kEgWaves = kEgBlock / 64;
constexpr int kScanChunk = 4096;              // cubes per scan block (16 per thread)
constexpr int kEgMaxWords = 64 * 8 * 63 / 32 + 2;  // worst cube: 512 codes of 63 bits, plus alignment

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

// block b: sum of bits over its chunk of kScanChunk cubes
__global__ __launch_bounds__(kEgBlock) void eg_scan_reduce_kernel(EgParams P) {
    __shared__ uint64_t part[kEgWaves];
    const uint64_t base = (uint64_t)blockIdx.x * kScanChunk + threadIdx.x * (kScanChunk / kEgBlock);
    uint64_t s = 0;
    for (int i = 0; i < kScanChunk / kEgBlock; i++)
        if (base + i < P.n_cubes) s += P.bits[base + i];
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

// block b: per-cube exclusive offsets inside the chunk, plus the chunk's offset
__global__ __launch_bounds__(kEgBlock) void eg_scan_apply_kernel(EgParams P) {
    constexpr int PER = kScanChunk / kEgBlock;
    __shared__ uint64_t part[kEgBlock];
    const uint64_t base = (uint64_t)blockIdx.x * kScanChunk + threadIdx.x * PER;
    uint32_t v[PER];
    uint64_t s = 0;
#pragma unroll
    for (int i = 0; i < PER; i++) {
        v[i] = base + i < P.n_cubes ? P.bits[base + i] : 0u;
        s += v[i];
    }
    part[threadIdx.x] = s;
    __syncthreads();
    for (int o = 1; o < kEgBlock; o <<= 1) {
        const uint64_t t = threadIdx.x >= (unsigned)o ? part[threadIdx.x - o] : 0;
        __syncthreads();
        part[threadIdx.x] += t;
        __syncthreads();
    }
    uint64_t run = P.bsum[blockIdx.x] + part[threadIdx.x] - s;
#pragma unroll
    for (int i = 0; i < PER; i++) {
        if (base + i < P.n_cubes) P.off[base + i] = run;
        run += v[i];
    }
}

// clears the words the stream will occupy; word 0 keeps the carried partial byte (stream byte 0)
__global__ __launch_bounds__(kEgBlock) void eg_zero_kernel(EgParams P) {
    if (P.status[1] != 0) return;
    const uint64_t words = (P.status[0] + 31) / 32;
    for (uint64_t w = (uint64_t)blockIdx.x * kEgBlock + threadIdx.x; w < words; w += (uint64_t)gridDim.x * kEgBlock)
        P.out[w] = w == 0 ? (uint32_t)(P.carry_byte & (0xFF00u >> P.carry_bits)) : 0u;
}

template <int D>
__global__ __launch_bounds__(kEgBlock) void eg_write_kernel(EgParams P) {
    constexpr int CS = 64 * D, PER = CS / 64;
    __shared__ int32_t sq[kEgWaves][CS];
    __shared__ uint32_t img[kEgWaves][kEgMaxWords];
    if (P.status[1] != 0) return;  // capacity or range failure: nothing is written
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t g = (uint64_t)blockIdx.x * kEgWaves + wave;
    if (g >= P.n_cubes) return;
    // stage the cube (coalesced), then read it in diagonal-slice order
    const int32_t* q = P.q + g * CS;
#pragma unroll
    for (int i = 0; i < PER; i += 4) *(int4*)&sq[wave][(i / 4) * 256 + lane * 4] = *(const int4*)(q + (i / 4) * 256 + lane * 4);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    uint32_t code[PER];
    int width[PER];
    bool bad = false;
    uint32_t lbits = 0;
#pragma unroll
    for (int i = 0; i < PER; i++) {
        code[i] = eg_code(sq[wave][P.diag[lane * PER + i]], width[i], bad);
        lbits += (uint32_t)width[i];
    }
    // exclusive scan of the lanes' bit counts (stream order = lane order)
    uint32_t incl = lbits;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(incl, o, 64);
        if (lane >= o) incl += t;
    }
    const uint32_t total = __shfl(incl, 63, 64);
    const uint64_t start = P.off[g];
    const uint32_t s0 = (uint32_t)(start & 31);
    const uint64_t w0 = start >> 5;
    const uint32_t nwords = (s0 + total + 31) >> 5;
    for (uint32_t w = lane; w < nwords; w += 64) img[wave][w] = 0u;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    uint32_t pos = s0 + incl - lbits;  // stream bit of this lane's first code, relative to word w0
#pragma unroll
    for (int i = 0; i < PER; i++) {
        // the value occupies the last n bits of the code: stream bits [pos + width - n, pos + width)
        const uint32_t e = pos + (uint32_t)width[i];
        const uint32_t n = ((uint32_t)width[i] + 1) >> 1;
        const uint32_t kl = (e - 1) >> 5;
        const uint32_t r = e - 32 * kl;  // 1..32 bits of the value in word kl
        atomicOr(&img[wave][kl], r == 32 ? code[i] : code[i] << (32 - r));
        if (n > r) atomicOr(&img[wave][kl - 1], code[i] >> r);
        pos = e;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (uint32_t w = lane; w < nwords; w += 64) {
        const uint32_t v = __builtin_bswap32(img[wave][w]);  // stream order -> memory byte order
        if (w == 0 || w == nwords - 1) atomicOr(&P.out[w0 + w], v);  // shared with a neighbour
        else P.out[w0 + w] = v;
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
    hipLaunchKernelGGL(eg_zero_kernel, dim3(2048), dim3(kEgBlock), 0, st, P);
    if (D == 8) hipLaunchKernelGGL(eg_write_kernel<8>, dim3((uint32_t)cube_blocks), dim3(kEgBlock), 0, st, P);
    else hipLaunchKernelGGL(eg_write_kernel<4>, dim3((uint32_t)cube_blocks), dim3(kEgBlock), 0, st, P);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace dct3d
