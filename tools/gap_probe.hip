// Probe: the idle time between dependent kernels of one stream, launched one by one vs replayed from a
// hipGraph.  A write-heavy kernel (512 MiB of 16-byte stores, like the stream decode's raster) alternates
// with a small one (a 2,048-block kernel that writes one word per block, like the scan kernels);
// the time of N pairs is compared with the kernels alone.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/gap_probe tools/gap_probe.hip && /tmp/gap_probe [stream|graph]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

__global__ __launch_bounds__(256) void big_write(uint4* p, size_t n, uint32_t v) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
        p[i] = make_uint4(v, v + 1, v + 2, (uint32_t)i);
}
__global__ __launch_bounds__(256) void small(uint32_t* q, uint32_t v) {
    if (threadIdx.x == 0) q[blockIdx.x] = v + blockIdx.x;
}

int main(int argc, char** argv) {
    const bool only_graph = argc > 1 && argv[1][0] == 'g', only_stream = argc > 1 && argv[1][0] == 's';
    const size_t bytes = 512ull << 20, n = bytes / 16;
    uint4* p;
    uint32_t* q;
    CK(hipMalloc(&p, bytes));
    CK(hipMalloc(&q, 2048 * 4));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const int N = 20;
    auto pairs = [&](hipStream_t st, int mode) {  // mode 0: pairs, 1: big only, 2: small only
        for (int i = 0; i < N; i++) {
            if (mode != 2) hipLaunchKernelGGL(big_write, dim3(4096), dim3(256), 0, st, p, n, (uint32_t)i);
            if (mode != 1) hipLaunchKernelGGL(small, dim3(2048), dim3(256), 0, st, q, (uint32_t)i);
        }
    };
    auto timed = [&](auto&& body) {
        body();  // warm
        CK(hipStreamSynchronize(s));
        CK(hipEventRecord(a, s));
        for (int r = 0; r < 5; r++) body();
        CK(hipEventRecord(b, s));
        CK(hipEventSynchronize(b));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, a, b));
        return ms * 1e3f / (5 * N);  // us per iteration
    };
    float t_pair = 0.f, t_big = 0.f, t_small = 0.f, t_graph = 0.f;
    if (!only_graph) {
        t_pair = timed([&] { pairs(s, 0); });
        t_big = timed([&] { pairs(s, 1); });
        t_small = timed([&] { pairs(s, 2); });
    }
    if (!only_stream) {
        hipGraph_t g;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        pairs(s, 0);
        CK(hipStreamEndCapture(s, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        t_graph = timed([&] { CK(hipGraphLaunch(ge, s)); });
    }
    printf("{\"stream_pair_us\": %.2f, \"big_only_us\": %.2f, \"small_only_us\": %.2f, \"graph_pair_us\": %.2f}\n",
           t_pair, t_big, t_small, t_graph);
    return 0;
}
