// dct3d_diag.hip -- libdct3d_diag.so: measurement and test support, NOT the product path.
//
// Everything here exists to measure or to feed the product kernels (libdct3d.so), and nothing in the
// product calls it:
//   * memory-only twins of the encode kernels (the same loads, LDS staging and 1 KiB NT stores,
//     without the transform): the ceiling the encode's own traffic reaches (bench.py "ceiling");
//   * the decode kernel split into memory only (no transform) and compute only (no global loads, no
//     stores), so its time can be read against both;
//   * a bandwidth probe of plain traffic mixes (1:4 read/write, copy, write-only, read-only);
//   * the deterministic synthetic frames the bench and the GPU tests encode.
// The twins instantiate the product's own device templates (dct3d_encode_dev.h, dct3d_decode_dev.h)
// with the transform switched off, so their memory behaviour is the product's.  C-ABI:
// include/dct3d_diag.h.
#include <cmath>
#include <cstring>
#include <mutex>
#include <vector>

#include "dct3d.h"
#include "dct3d_diag.h"
#include "dct3d_decode_dev.h"
#include "dct3d_encode_dev.h"

namespace dct3d {

// 8x8x4 twin (dct3d_encode_memonly_dev; the output is NOT a DCT): the encode's memory traffic alone --
// the same row loads, the same LDS staging and 1 KiB NT stores of 16 KiB per wave -- with the
// transform, quantisation and certification replaced by a few integer ops on the loaded bytes.  Its
// rate is the ceiling the encode's own traffic reaches on this device (bench.py: ceiling).
template <int D>
__global__ __launch_bounds__(kBlock, 4) void encode_memonly_kernel(EncodeParams P) {
    __shared__ __attribute__((aligned(16))) char lds[kWavesPerBlock * enc_wave_lds<D>()];
    constexpr int NB = (D == 8) ? 8 : 4;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t cube0 = P.g_base + (xcd_tile<64>() * kWavesPerBlock + wave) * kCubesPerWave;  // the product's order
    uint2 raw[D];
    load_rows<D>(P, cube0 + (lane >> 3), cube0 + (lane >> 3) < P.n_cubes, lane & 7, raw);
    if (cube0 >= P.n_cubes) return;
    int32_t qv[8][NB];
#pragma unroll
    for (int ky = 0; ky < 8; ky++)
#pragma unroll
        for (int x = 0; x < NB; x++) qv[ky][x] = (int32_t)((ky & 1 ? raw[x % D].y : raw[x % D].x) >> (ky * 3 % 24)) & 255;
    enc_stage_store<D, true>(P, qv, lds + wave * enc_wave_lds<D>(), lane, cube0);
}

// dct3d_decode_diag_dev (the output is NOT a decode): MODE 1 = memory only
// (the same loads, staging and raster stores, no transform), MODE 2 = compute only (no global loads;
// stores suppressed by a runtime condition).  They split the kernel's time into its memory and compute
// parts (1.9 ms / 1.8 ms against 2.25 ms for the full kernel, c3).
template <int D, int MODE>
__global__ __launch_bounds__(kBlock, 4) void decode_kernel_diag(DecodeParams P) {
    __shared__ __attribute__((aligned(16))) char lds[kWavesPerBlock * kDecWaveLds];
    using G = DecGeom<D>;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    char* wl = lds + wave * kDecWaveLds;
    const uint32_t cube0 = (xcd_tile() * kWavesPerBlock + wave) * G::CPW;  // the product's order
    int4 v[8];
    if (MODE == 2) {
        for (int t = 0; t < 8; t++) v[t] = make_int4(lane + t, (int)cube0 & 7, t, 1);
    } else {
        dec_load_tile<D>(P, cube0, lane, v);
    }
    dec_stage_tile<D>(wl, lane, v);
    wave_lds_sync();
    if (MODE == 1) {  // the product's loads, staging reads and stores (dec_store_tile), no transform
        const int h = (lane >> 4) & 1, k = lane & (D - 1);
        const int c = (lane >> 5) * (G::CPW / 2) + ((lane & 15) / D);
        uint32_t acc = 0;
        for (int ky = 0; ky < 8; ky++) {
            const int4 x = *(const int4*)(wl + c * G::SA_C + k * G::SA_F + h * 16 + ky * 32);
            acc += x.x ^ x.y ^ x.z ^ x.w;
        }
        uint32_t outw[D][(D == 8) ? 1 : 2];
#pragma unroll
        for (int z = 0; z < D; z++)
#pragma unroll
            for (int wd = 0; wd < ((D == 8) ? 1 : 2); wd++) outw[z][wd] = acc + z + wd;
        wave_lds_sync();
        dec_store_tile<D>(P, wl, lane, cube0, outw, cube0 + c < P.n_cubes);
        return;
    }
    DecodeParams Q = P;
    if (MODE == 2 && P.width != 0xFFFFFFFFu) Q.n_cubes = 0;  // all stores suppressed, compute kept
    decode_tile<D, 1>(Q, wl, lane, cube0, [] {}, ReloadCubes<D>{P.in});
}

// =============================================================================================
// Synthetic frames (integer-only, reproducible on host)
// =============================================================================================
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    uint64_t z = x;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void synth_kernel(uint8_t* out, int width, int height, long long n_pix, uint64_t seed,
                                                     long long frame0, int kind) {
    const long long plane = (long long)width * height;
    for (long long base = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 16; base < n_pix;
         base += (long long)gridDim.x * blockDim.x * 16) {
        uint32_t w[4] = {0, 0, 0, 0};
        for (int i = 0; i < 16 && base + i < n_pix; i++) {
            const long long p = base + i;
            const long long f = p / plane + frame0;
            const long long rem = p % plane;
            const int y = (int)(rem / width), x = (int)(rem % width);
            const uint64_t idx = (uint64_t)(frame0 * plane + p);
            const uint64_t h = splitmix64(seed ^ idx);
            int v;
            if (kind == 1) v = (int)(h & 255u);
            else {
                v = 128 + (int)((3ll * x + 5ll * y + 7ll * f) & 63) - 32 + (int)(h & 15u);
                v = v < 0 ? 0 : (v > 255 ? 255 : v);
            }
            w[i >> 2] |= (uint32_t)v << (8 * (i & 3));
        }
        if (base + 16 <= n_pix) {
            *(uint4*)(out + base) = make_uint4(w[0], w[1], w[2], w[3]);
        } else {
            for (int i = 0; base + i < n_pix; i++) out[base + i] = (uint8_t)(w[i >> 2] >> (8 * (i & 3)));
        }
    }
}

// =============================================================================================
// Bandwidth calibration: the encode's traffic mix without the transform.  mode 0: read n_px bytes,
// write 4*n_px (1:4, NT); mode 1: copy (NT); mode 2: write-only 4*n_px (NT); mode 3: read-only.
// =============================================================================================
__global__ __launch_bounds__(256) void ceiling_kernel(const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                                       long long n_px, int mode, unsigned* sink) {
    // Pure streaming, every wave-instruction a contiguous 1 KiB: per iteration a thread reads 4
    // 16-byte chunks (4 loads in flight) and writes 16 (mix 1:4), 4 (copy) or 16 (write-only).
    const long long T = (long long)gridDim.x * blockDim.x;
    const long long g = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long n_in = n_px / 16;
    unsigned acc = 0;
    for (long long it = 0; it * 4 * T < n_in; it++) {
        uint4 v[4];
        if (mode != 2 && mode != 5) {
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const long long c = it * 4 * T + u * T + g;
                if (c < n_in) {
                    const i32x4_t t = __builtin_nontemporal_load((const i32x4_t*)(in + c * 16));
                    v[u] = make_uint4((unsigned)t.x, (unsigned)t.y, (unsigned)t.z, (unsigned)t.w);
                } else {
                    v[u] = make_uint4(0, 0, 0, 0);
                }
            }
        } else {
#pragma unroll
            for (int u = 0; u < 4; u++) v[u] = make_uint4((unsigned)it, (unsigned)g, u, 0);
        }
        if (mode == 0 || mode == 2) {
#pragma unroll
            for (int w = 0; w < 16; w++) {
                const long long o = it * 16 * T + w * T + g;
                const uint4 x = v[w & 3];
                if (o < 4 * n_in) store16<true>(out + o * 16, make_int4((int)x.x, (int)x.y, (int)x.z, (int)(x.w + w)));
            }
        } else if (mode == 1 || mode == 4) {
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const long long c = it * 4 * T + u * T + g;
                const int4 o = make_int4((int)v[u].x, (int)v[u].y, (int)v[u].z, (int)v[u].w);
                if (c < n_in) {
                    if (mode == 1) store16<true>(out + c * 16, o);
                    else *(int4*)(out + c * 16) = o;
                }
            }
        } else if (mode == 5) {
#pragma unroll
            for (int w = 0; w < 16; w++) {
                const long long o = it * 16 * T + w * T + g;
                if (o < 4 * n_in) *(int4*)(out + o * 16) = make_int4((int)it, (int)g, w, 0);
            }
        } else {
#pragma unroll
            for (int u = 0; u < 4; u++) acc += v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
        }
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

static int launch_ceiling(const uint8_t* in, uint8_t* out, long long n_px, int mode, unsigned* sink, hipStream_t st) {
    static int grid = -1;
    if (grid < 0) {
        const char* e = getenv("DCT3D_PROBE_GRID");  // calibration knob: blocks of 256 threads
        grid = e ? atoi(e) : 16384;  // best of the 1024..16384 sweep (profiles/r01/probe_sweep.txt)
    }
    hipLaunchKernelGGL(ceiling_kernel, dim3(grid), dim3(256), 0, st, in, out, n_px, mode, sink);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

namespace {

FastDiv fast_div(uint32_t d) {  // as dct3d_runtime.cpp: s = 31 + ceil(log2 d), m = ceil(2^s / d)
    uint32_t l = 0;
    while ((1ull << l) < d) l++;
    FastDiv f;
    f.s = 31 + l;
    f.m = (uint32_t)(((1ull << f.s) + d - 1) / d);
    return f;
}

struct CtxView {
    int device = 0, bd = 8;
    hipStream_t stream = nullptr;
};
int view(dct3d_ctx* c, CtxView& v) {
    void* st = nullptr;
    if (!c || dct3d_ctx_info(c, &v.device, &v.bd, &st) != DCT3D_OK) return DCT3D_EINVAL;
    v.stream = (hipStream_t)st;
    return hipSetDevice(v.device) == hipSuccess ? DCT3D_OK : DCT3D_EDEVICE;
}
int geometry(int w, int h, int n_stacks, uint64_t* n_cubes) {
    if (w <= 0 || h <= 0 || n_stacks < 0 || w % 8 || h % 8) return DCT3D_EINVAL;
    const uint64_t n = (uint64_t)(w / 8) * (uint64_t)(h / 8) * (uint64_t)n_stacks;
    if (n >= (1ull << 31) / 8) return DCT3D_EINVAL;
    *n_cubes = n;
    return DCT3D_OK;
}

// Per-device scratch of the diagnostics (grown, never freed: a diagnostic library), allocated before
// any timed launch so that a call never waits on an allocation between its caller's events.
struct Scratch {
    void* p = nullptr;
    size_t bytes = 0;
};
std::mutex g_mu;
Scratch g_scratch[64];
void* scratch(int device, size_t bytes) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (device < 0 || device >= 64) return nullptr;
    Scratch& s = g_scratch[device];
    if (s.bytes < bytes) {
        if (s.p) (void)hipFree(s.p);
        s.p = nullptr;
        s.bytes = 0;
        if (hipMalloc(&s.p, bytes) != hipSuccess) return nullptr;
        if (hipMemset(s.p, 0, bytes) != hipSuccess) return nullptr;
        s.bytes = bytes;
    }
    return s.p;
}

// The 8x8x8 encode's tables on the device for the compute-only twin (its certificate, second
// certificate and Java fold tables, from dct3d_plan_query; the second certificate's basis from the cosine
// directly: the twin's output is discarded, only its work matters).  Built once per device.
constexpr int kMaxS = 32;  // the plan's per-s table size (dct3d_plan.h, dct3d_plan_info)
struct EncTables {
    float* tabs = nullptr;  // [3 * kMaxS] 1/step, G, E
    double* tab64 = nullptr;
    int32_t* ngroups = nullptr;
    double* coef = nullptr;
    uint8_t* group_of = nullptr;
    double coef_dc = 0.0;
};
EncTables g_enc8[64];
const EncTables* enc8_tables(int device) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (device < 0 || device >= 64) return nullptr;
    EncTables& t = g_enc8[device];
    if (t.tabs) return &t;
    constexpr int CS = 512;
    dct3d_plan_info info;
    std::vector<int32_t> ng(CS);
    std::vector<double> cf((size_t)CS * kMaxGroupsDev);
    std::vector<uint8_t> go((size_t)CS * CS);
    if (dct3d_plan_query(8, 8, 8, &info, ng.data(), cf.data(), go.data(), nullptr) != DCT3D_OK) return nullptr;
    float tabs[3 * kMaxS];
    memcpy(tabs, info.enc_rstep, sizeof(float) * kMaxS);
    memcpy(tabs + kMaxS, info.enc_G, sizeof(float) * kMaxS);
    memcpy(tabs + 2 * kMaxS, info.enc_E, sizeof(float) * kMaxS);
    double t64[64 + kMaxS];
    for (int kk = 0; kk < 8; kk++)
        for (int n = 0; n < 8; n++)
            t64[kk * 8 + n] = (kk ? 0.5 : std::sqrt(0.125)) * std::cos((2 * n + 1) * kk * 3.14159265358979323846 / 16);
    memcpy(t64 + 64, info.enc_thr64, sizeof(double) * kMaxS);
    EncTables n;
    if (hipMalloc((void**)&n.tabs, sizeof(tabs)) != hipSuccess || hipMalloc((void**)&n.tab64, sizeof(t64)) != hipSuccess ||
        hipMalloc((void**)&n.ngroups, ng.size() * 4) != hipSuccess || hipMalloc((void**)&n.coef, cf.size() * 8) != hipSuccess ||
        hipMalloc((void**)&n.group_of, go.size()) != hipSuccess ||
        hipMemcpy(n.tabs, tabs, sizeof(tabs), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(n.tab64, t64, sizeof(t64), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(n.ngroups, ng.data(), ng.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(n.coef, cf.data(), cf.size() * 8, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(n.group_of, go.data(), go.size(), hipMemcpyHostToDevice) != hipSuccess)
        return nullptr;
    n.coef_dc = info.coef_dc;
    t = n;
    return &t;
}

}  // namespace
}  // namespace dct3d

using namespace dct3d;

extern "C" {

int dct3d_fill_synthetic_dev(dct3d_ctx* c, uint8_t* d, int w, int h, int n_frames, uint64_t seed, int64_t frame0,
                             int kind) {
    CtxView v;
    if (!d || w <= 0 || h <= 0 || n_frames < 0 || (kind != 0 && kind != 1)) return DCT3D_EINVAL;
    int rc = view(c, v);
    if (rc) return rc;
    const long long n_pix = (long long)w * h * n_frames;
    long long blocks = ((n_pix + 15) / 16 + 255) / 256;
    blocks = blocks > 65536 ? 65536 : (blocks < 1 ? 1 : blocks);
    hipLaunchKernelGGL(synth_kernel, dim3((unsigned)blocks), dim3(256), 0, v.stream, d, w, h, n_pix, seed, frame0, kind);
    return hipGetLastError() == hipSuccess ? DCT3D_OK : DCT3D_EKERNEL;
}

int dct3d_bandwidth_probe_dev(dct3d_ctx* c, const uint8_t* d_in, void* d_out, size_t n_px, int mode) {
    CtxView v;
    if (n_px % 16 || mode < 0 || mode > 5 || (mode != 2 && mode != 5 && !d_in) || (mode != 3 && !d_out))
        return DCT3D_EINVAL;
    int rc = view(c, v);
    if (rc) return rc;
    unsigned* sink = (unsigned*)scratch(v.device, 64);
    if (!sink) return DCT3D_ENOMEM;
    return launch_ceiling(d_in, (uint8_t*)d_out, (long long)n_px, mode, sink, v.stream) ? DCT3D_EKERNEL : DCT3D_OK;
}

int dct3d_encode_memonly_dev(dct3d_ctx* c, const uint8_t* d_raster, int w, int h, int n_stacks, int32_t* d_q) {
    return dct3d_encode_diag_dev(c, d_raster, w, h, n_stacks, d_q, 1);
}

int dct3d_encode_diag_dev(dct3d_ctx* c, const uint8_t* d_raster, int w, int h, int n_stacks, int32_t* d_q, int mode) {
    return dct3d_encode_trace_dev(c, d_raster, w, h, n_stacks, d_q, mode, nullptr);
}

static int encode_diag(dct3d_ctx* c, const uint8_t* d_raster, int w, int h, int n_stacks, int32_t* d_q, int mode,
                       uint64_t* d_trace, int strip_w);
int dct3d_encode_trace_dev(dct3d_ctx* c, const uint8_t* d_raster, int w, int h, int n_stacks, int32_t* d_q, int mode,
                           uint64_t* d_trace) {
    return encode_diag(c, d_raster, w, h, n_stacks, d_q, mode, d_trace, 0);
}

int dct3d_encode_strip_dev(dct3d_ctx* c, const uint8_t* d_raster, int w, int h, int n_stacks, int32_t* d_q, int mode,
                           int strip_w) {
    if ((mode != 0 && mode != 1) || strip_w <= 0 || strip_w % 4 || w <= 0 || (w / 8) % strip_w) return DCT3D_EINVAL;
    return encode_diag(c, d_raster, w, h, n_stacks, d_q, mode == 1 ? 4 : 5, nullptr, strip_w);
}

static int encode_diag(dct3d_ctx* c, const uint8_t* d_raster, int w, int h, int n_stacks, int32_t* d_q, int mode,
                       uint64_t* d_trace, int strip_w) {
    CtxView v;
    if ((!d_raster || !d_q) && n_stacks) return DCT3D_EINVAL;
    int rc = view(c, v);
    uint64_t n_cubes = 0;
    if (rc || (rc = geometry(w, h, n_stacks, &n_cubes))) return rc;
    if (mode != 1 && !((mode >= 2 && mode <= 5) && v.bd == 8)) return DCT3D_EINVAL;
    if (mode == 3 && !d_trace) return DCT3D_EINVAL;
    if (n_cubes == 0) return DCT3D_OK;
    EncodeParams P;
    memset(&P, 0, sizeof(P));
    P.raster = d_raster;
    P.out = d_q;
    P.n_cubes = (uint32_t)n_cubes;
    P.cubes_per_stack = (uint32_t)((w / 8) * (h / 8));
    P.nbx = (uint32_t)(w / 8);
    P.div_cps = fast_div(P.cubes_per_stack);
    P.div_nbx = fast_div(P.nbx);
    P.width = (uint32_t)w;
    P.plane = (uint64_t)w * h;
    P.stack_stride = P.plane * v.bd;
    if (strip_w) {
        P.strip_w = (uint32_t)strip_w;
        P.strip_cubes = (uint32_t)strip_w * (uint32_t)(h / 8);
        P.div_strip_w = fast_div(P.strip_w);
        P.div_strip_cubes = fast_div(P.strip_cubes);
    }
    if (v.bd == 8) {  // the twins of encode16_kernel
        const uint32_t groups = (P.n_cubes + kE16CPW - 1) / kE16CPW;
        const dim3 grid((groups + kWavesPerBlock - 1) / kWavesPerBlock);
        if (mode == 1 || mode == 4) {
            if (mode == 1) hipLaunchKernelGGL((encode16_kernel<true, 1>), grid, dim3(kBlock), 0, v.stream, P);
            else hipLaunchKernelGGL((encode16_kernel<true, 4>), grid, dim3(kBlock), 0, v.stream, P);
        } else {  // compute only / the product with the strip traversal, with the product's tables
            const EncTables* t = enc8_tables(v.device);
            if (!t) return DCT3D_ENOMEM;
            P.coef_dc = t->coef_dc;
            P.tab_rstep = t->tabs;
            P.tab_G = t->tabs + kMaxS;
            P.tab_E = t->tabs + 2 * kMaxS;
            P.tab64 = t->tab64;
            P.recheck = 1u;
            P.ngroups = t->ngroups;
            P.coef = t->coef;
            P.group_of = t->group_of;
            P.trace = d_trace;
            if (mode == 2) hipLaunchKernelGGL((encode16_kernel<true, 2>), grid, dim3(kBlock), 0, v.stream, P);
            else if (mode == 3) hipLaunchKernelGGL((encode16_kernel<true, 3>), grid, dim3(kBlock), 0, v.stream, P);
            else hipLaunchKernelGGL((encode16_kernel<true, 5>), grid, dim3(kBlock), 0, v.stream, P);
        }
    } else {
        const uint32_t groups = (P.n_cubes + kCubesPerWave - 1) / kCubesPerWave;
        hipLaunchKernelGGL((encode_memonly_kernel<4>), dim3((groups + kWavesPerBlock - 1) / kWavesPerBlock),
                           dim3(kBlock), 0, v.stream, P);
    }
    return hipGetLastError() == hipSuccess ? DCT3D_OK : DCT3D_EKERNEL;
}

int dct3d_decode_diag_dev(dct3d_ctx* c, const int32_t* d_q, int w, int h, int n_stacks, uint8_t* d_raster, int mode) {
    CtxView v;
    if ((mode != 1 && mode != 2) || ((!d_q || !d_raster) && n_stacks)) return DCT3D_EINVAL;
    int rc = view(c, v);
    uint64_t n_cubes = 0;
    if (rc || (rc = geometry(w, h, n_stacks, &n_cubes))) return rc;
    if (n_cubes == 0) return DCT3D_OK;
    DecodeParams P;
    memset(&P, 0, sizeof(P));
    P.in = d_q;
    P.out = d_raster;
    P.n_cubes = (uint32_t)n_cubes;
    P.cubes_per_stack = (uint32_t)((w / 8) * (h / 8));
    P.nbx = (uint32_t)(w / 8);
    P.div_cps = fast_div(P.cubes_per_stack);
    P.div_nbx = fast_div(P.nbx);
    P.width = (uint32_t)w;
    P.plane = (uint64_t)w * h;
    P.stack_stride = P.plane * v.bd;
    P.blk_store = mode == 1 && P.nbx % 2 == 0 && P.stack_stride < (1ull << 32) ? 1u : 0u;  // as the product (mode 2 stores nothing)
    P.inv_coef_t = nullptr;  // no replay: mode 1 certifies nothing, mode 2 stores (and so flags) nothing
    const uint32_t per = (v.bd == 8 ? DecGeom<8>::CPW : DecGeom<4>::CPW) * kWavesPerBlock;
    const uint32_t groups = (uint32_t)((n_cubes + per - 1) / per);
    if (v.bd == 8) {
        if (mode == 1) hipLaunchKernelGGL((decode_kernel_diag<8, 1>), dim3(groups), dim3(kBlock), 0, v.stream, P);
        else hipLaunchKernelGGL((decode_kernel_diag<8, 2>), dim3(groups), dim3(kBlock), 0, v.stream, P);
    } else {
        if (mode == 1) hipLaunchKernelGGL((decode_kernel_diag<4, 1>), dim3(groups), dim3(kBlock), 0, v.stream, P);
        else hipLaunchKernelGGL((decode_kernel_diag<4, 2>), dim3(groups), dim3(kBlock), 0, v.stream, P);
    }
    return hipGetLastError() == hipSuccess ? DCT3D_OK : DCT3D_EKERNEL;
}

}  // extern "C"
