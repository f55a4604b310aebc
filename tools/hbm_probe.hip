// hbm_probe.hip -- standalone HBM write / mixed-traffic probe (tool, not part of the product library).
// Measures how store shape, cache policy, per-wave contiguity and occupancy change the achievable
// rate for the encode kernel's traffic: 1 B/px read, 4 B/px written (4,147,200 cubes per step).
//   build: hipcc --offload-arch=gfx950 -O3 -o tools/bin/hbm_probe tools/hbm_probe.hip
//   run:   tools/bin/hbm_probe   (prints one line per configuration)
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

typedef int i32x4 __attribute__((ext_vector_type(4)));

// each wave owns `chunk` output bytes (and chunk/4 input bytes when READ): 16 B per lane per
// instruction, W_ITERS instructions per wave = chunk / 1024
template <bool NT, bool READ, bool DWORD>
__global__ __launch_bounds__(256) void wave_chunk(const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                                  uint64_t chunk, uint64_t n_chunks) {
    const uint64_t wave = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (wave >= n_chunks) return;
    int acc = 0;
    if (READ) {
        const uint8_t* src = in + wave * (chunk / 4);
        for (uint64_t o = lane * 16; o < chunk / 4; o += 1024) {
            const i32x4 v = NT ? __builtin_nontemporal_load((const i32x4*)(src + o)) : *(const i32x4*)(src + o);
            acc += v.x ^ v.y ^ v.z ^ v.w;
        }
    }
    uint8_t* dst = out + wave * chunk;
    if (DWORD) {
        for (uint64_t o = lane * 4; o < chunk; o += 256) {
            if (NT) __builtin_nontemporal_store(acc + (int)o, (int*)(dst + o));
            else *(int*)(dst + o) = acc + (int)o;
        }
    } else {
        for (uint64_t o = lane * 16; o < chunk; o += 1024) {
            const i32x4 v = {acc, (int)o, lane, 1};
            if (NT) __builtin_nontemporal_store(v, (i32x4*)(dst + o));
            else *(i32x4*)(dst + o) = v;
        }
    }
}

template <bool NT, bool READ, bool DWORD>
float run(const uint8_t* in, uint8_t* out, uint64_t bytes, uint64_t chunk, int lds_kb, int reps) {
    const uint64_t n_chunks = bytes / chunk;
    const uint64_t blocks = (n_chunks + 3) / 4;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    hipLaunchKernelGGL((wave_chunk<NT, READ, DWORD>), dim3((uint32_t)blocks), dim3(256), lds_kb * 1024, 0, in, out, chunk,
                       n_chunks);
    (void)hipEventRecord(a, 0);
    for (int r = 0; r < reps; r++)
        hipLaunchKernelGGL((wave_chunk<NT, READ, DWORD>), dim3((uint32_t)blocks), dim3(256), lds_kb * 1024, 0, in, out,
                           chunk, n_chunks);
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms / reps;
}

int main() {
    const uint64_t out_bytes = 4147200ull * 2048;  // 8.49 GB: the encode's int32 output per step
    uint8_t *in = nullptr, *out = nullptr;
    if (hipMalloc(&in, out_bytes / 4 + (1 << 20)) != hipSuccess || hipMalloc(&out, out_bytes + (1 << 20)) != hipSuccess) {
        printf("alloc failed\n");
        return 1;
    }
    (void)hipMemset(in, 1, out_bytes / 4);
    (void)hipMemset(out, 0, out_bytes);
    const int reps = 5;
    printf("mode read chunkKiB ldsKiB(occupancy) ms TB/s(total bytes)\n");
    const uint64_t chunks[] = {16384, 65536, 262144};
    const int ldss[] = {0, 20, 40, 80};  // 0: 32 waves/CU max, 20 KiB: 8 blocks.., 40: 4 blocks, 80: 2 blocks
    for (int read = 0; read < 2; read++)
        for (uint64_t ch : chunks)
            for (int lds : ldss) {
                const double tot = (double)out_bytes * (read ? 1.25 : 1.0);
                float ms;
                ms = read ? run<true, true, false>(in, out, out_bytes, ch, lds, reps)
                          : run<true, false, false>(in, out, out_bytes, ch, lds, reps);
                printf("nt_x4   %d %6llu %3d %8.3f %6.2f\n", read, (unsigned long long)(ch / 1024), lds, ms, tot / ms / 1e9);
                ms = read ? run<false, true, false>(in, out, out_bytes, ch, lds, reps)
                          : run<false, false, false>(in, out, out_bytes, ch, lds, reps);
                printf("pl_x4   %d %6llu %3d %8.3f %6.2f\n", read, (unsigned long long)(ch / 1024), lds, ms, tot / ms / 1e9);
                ms = read ? run<false, true, true>(in, out, out_bytes, ch, lds, reps)
                          : run<false, false, true>(in, out, out_bytes, ch, lds, reps);
                printf("pl_dw   %d %6llu %3d %8.3f %6.2f\n", read, (unsigned long long)(ch / 1024), lds, ms, tot / ms / 1e9);
                fflush(stdout);
            }
    return 0;
}
