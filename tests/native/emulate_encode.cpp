// tests/native/emulate_encode.cpp -- TEST ONLY: host emulation of the fused encode kernel's fp32
// arithmetic (csrc/dct3d_kernels.hip, encode_kernel): the same butterfly source
// (csrc/dct_butterfly.h) in the same order -- pass X with the exact integer front and cube-mean
// centring, pass Z, pass Y -- then the kernel's quantise/certify step.  Built by the tests with
// g++ -O2 -ffp-contract=off; never linked into the product.
#include <cmath>
#include <cstdint>
#include <cstring>

#include "dct_butterfly.h"

using namespace dct3d;

extern "C" int emulate_encode(const uint8_t* cubes, int n_cubes, int D, const float* rstep, const float* G,
                              const float* E, double coef_dc, int32_t* q_out, uint8_t* flag_out, float* val_out,
                              float* A_out) {
    const int CS = 64 * D;
    for (int g = 0; g < n_cubes; g++) {
        const uint8_t* x = cubes + (size_t)g * CS;
        uint32_t S = 0, mx = 0, mn = 255;
        for (int i = 0; i < CS; i++) {
            S += x[i];
            mx = x[i] > mx ? x[i] : mx;
            mn = x[i] < mn ? x[i] : mn;
        }
        const int m = (int)((S + CS / 2) / CS);
        const float A = std::fmax((float)mx - (float)m, (float)m - (float)mn);
        float v[8][8][8];  // [z][y][x]
        for (int z = 0; z < D; z++)
            for (int y = 0; y < 8; y++)
                for (int xx = 0; xx < 8; xx++) v[z][y][xx] = (float)x[(z * 8 + y) * 8 + xx];
        const float dcsub = 8.0f * (float)m;
        for (int z = 0; z < D; z++)
            for (int y = 0; y < 8; y++) fdct8<true, true>(v[z][y], dcsub);
        for (int y = 0; y < 8; y++)
            for (int xx = 0; xx < 8; xx++) {
                if (D == 8) {
                    float col[8];
                    for (int z = 0; z < 8; z++) col[z] = v[z][y][xx];
                    fdct8<false, false>(col, 0.f);
                    for (int z = 0; z < 8; z++) v[z][y][xx] = col[z];
                } else {
                    float col[4];
                    for (int z = 0; z < 4; z++) col[z] = v[z][y][xx];
                    fdct4<false, false>(col, 0.f);
                    for (int z = 0; z < 4; z++) v[z][y][xx] = col[z];
                }
            }
        for (int z = 0; z < D; z++)
            for (int xx = 0; xx < 8; xx++) {
                float col[8];
                for (int y = 0; y < 8; y++) col[y] = v[z][y][xx];
                fdct8<false, false>(col, 0.f);
                for (int y = 0; y < 8; y++) v[z][y][xx] = col[y];
            }
        A_out[g] = A;
        for (int kz = 0; kz < D; kz++)
            for (int ky = 0; ky < 8; ky++)
                for (int kx = 0; kx < 8; kx++) {
                    const int k = (kz * 8 + ky) * 8 + kx, s = kx + ky + kz;
                    const float thr = std::fma(-A, G[s], 0.5f - E[s]);
                    const float q = v[kz][ky][kx] * rstep[s];
                    const float n = std::rint(q);
                    val_out[(size_t)g * CS + k] = v[kz][ky][kx];
                    flag_out[(size_t)g * CS + k] = std::fabs(q - n) >= thr;
                    q_out[(size_t)g * CS + k] = (int32_t)n;
                }
        // exact DC (single Java group): JavaRound(S * coef_dc)
        const double p = (double)S * coef_dc;
        const double f = std::floor(p);
        q_out[(size_t)g * CS] = (int32_t)f + ((p - f) >= 0.5 ? 1 : 0);
        flag_out[(size_t)g * CS] = 0;
    }
    return 0;
}
