// The 8x8x8 encode's fp32 error bound (dct3d_plan.cpp's Tracked analysis of the kernel's butterflies)
// split by source: the mean bound over the coefficients with pass X, pass Z or the constants in exact
// (fp64-grade) arithmetic, as fractions of the kernel's bound.  DESIGN.md §4.
//   g++ -O2 -std=c++17 -I 3ddctvideoencoding_amd/csrc -I include tools/cert_pass_split.cpp -o /tmp/split && /tmp/split
#include "dct3d_plan.cpp"
#include <cstdio>
using namespace dct3d;
static std::vector<double> bound(double uX, double uZ, double uY, bool f32c) {
    const int D = 8, cs = 512;
    std::vector<Tracked> v(cs);
    for (int n = 0; n < cs; n++) { v[n] = Tracked(cs); v[n].w[n] = 1.0; }
    auto at = [&](int z, int y, int x) -> Tracked& { return v[(z * 8 + y) * 8 + x]; };
    Tracked zero(cs);
    g_f32 = f32c;
    g_u = uX;
    for (int z = 0; z < D; z++)
        for (int y = 0; y < 8; y++) {
            Tracked r[8];
            for (int x = 0; x < 8; x++) r[x] = at(z, y, x);
            fdct8<true, true>(r, zero);
            for (int x = 0; x < 8; x++) at(z, y, x) = r[x];
        }
    g_u = uZ;
    for (int y = 0; y < 8; y++)
        for (int x = 0; x < 8; x++) {
            Tracked r[8];
            for (int z = 0; z < 8; z++) r[z] = at(z, y, x);
            fdct8<false, false>(r, zero);
            for (int z = 0; z < 8; z++) at(z, y, x) = r[z];
        }
    g_u = uY;
    for (int z = 0; z < D; z++)
        for (int x = 0; x < 8; x++) {
            Tracked r[8];
            for (int y = 0; y < 8; y++) r[y] = at(z, y, x);
            fdct8<false, false>(r, zero);
            for (int y = 0; y < 8; y++) at(z, y, x) = r[y];
        }
    std::vector<double> K(cs);
    for (int k = 0; k < cs; k++) K[k] = v[k].e;
    return K;
}
static double mean(const std::vector<double>& K) {
    double s = 0;
    for (int k = 1; k < 512; k++) s += K[k];
    return s / 511;
}
int main() {
    const double u = std::ldexp(1.0, -24), u64 = std::ldexp(1.0, -53);
    const double full = mean(bound(u, u, u, true));
    printf("kernel bound (mean over k > 0): %.3e per unit max|x - m|\n", full);
    printf("pass X exact:          %.3f\n", mean(bound(u64, u, u, true)) / full);
    printf("passes X and Z exact:  %.3f\n", mean(bound(u64, u64, u, true)) / full);
    printf("constants exact:       %.3f\n", mean(bound(u, u, u, false)) / full);
    printf("constants only:        %.3f\n", mean(bound(0, 0, 0, true)) / full);
}
