// tests/native/emulate_decode.cpp -- TEST ONLY: host emulation of the decode kernel's fp64 arithmetic
// (csrc/dct3d_decode_dev.h, decode_tile): the exact dequantisation q * step, the per-cube L1 bound, then
// the same butterfly source (csrc/dct_butterfly.h) in the kernel's pass order -- inverse Y, X, Z --
// before the certificate; the last pass adds the fixed-point offset as the kernel does (idct8_fix) and
// the emulation subtracts it again (exactly: both lie in [2^20, 2^21)).  Built by the tests with g++ -O2 -ffp-contract=off; never linked into the
// product.
#include <algorithm>
#include <cmath>
#include <cstdint>

#include "dct_butterfly.h"

using namespace dct3d;

constexpr double kFix = 1572864.0;  // the kernel's fixed-point offset (kFixMagic), put in by the last pass

// q: cube-major int32 [n][D][8][8]; v_out: the kernel's fp64 values [n][D][8][8] (before the fixed-point
// add); l1_out: sum |q * step| per cube (exact up to the fp64 sum)
extern "C" int emulate_decode(const int32_t* q, int n_cubes, int D, double* v_out, double* l1_out) {
    const int CS = 64 * D;
    for (int g = 0; g < n_cubes; g++) {
        double b[8][8][8];  // [z][y][x]
        double l1 = 0.0;
        for (int z = 0; z < D; z++)
            for (int y = 0; y < 8; y++)
                for (int x = 0; x < 8; x++) {
                    const double st = (double)std::max(1, 5 * (x + y + z));
                    b[z][y][x] = (double)q[(size_t)g * CS + (z * 8 + y) * 8 + x] * st;
                    l1 += std::fabs(b[z][y][x]);
                }
        for (int z = 0; z < D; z++)
            for (int x = 0; x < 8; x++) {  // pass Y
                double r[8];
                for (int y = 0; y < 8; y++) r[y] = b[z][y][x];
                idct8(r);
                for (int y = 0; y < 8; y++) b[z][y][x] = r[y];
            }
        for (int z = 0; z < D; z++)
            for (int y = 0; y < 8; y++) {  // pass X
                double r[8];
                for (int x = 0; x < 8; x++) r[x] = b[z][y][x];
                idct8(r);
                for (int x = 0; x < 8; x++) b[z][y][x] = r[x];
            }
        for (int y = 0; y < 8; y++)
            for (int x = 0; x < 8; x++) {  // pass Z
                if (D == 8) {
                    double r[8];
                    for (int z = 0; z < 8; z++) r[z] = b[z][y][x];
                    idct8_fix(r, kFix);
                    for (int z = 0; z < 8; z++) b[z][y][x] = r[z];
                } else {
                    double r[4];
                    for (int z = 0; z < 4; z++) r[z] = b[z][y][x];
                    idct4_fix(r, kFix);
                    for (int z = 0; z < 4; z++) b[z][y][x] = r[z];
                }
            }
        for (int z = 0; z < D; z++)
            for (int y = 0; y < 8; y++)
                for (int x = 0; x < 8; x++) v_out[(size_t)g * CS + (z * 8 + y) * 8 + x] = b[z][y][x] - kFix;  // exact
        l1_out[g] = l1;
    }
    return 0;
}
