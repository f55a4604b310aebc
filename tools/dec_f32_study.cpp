// The fp32 certify-or-replay decode, measured on the host.  STUDY ONLY (never linked into
// the product).  The decode kernel runs its three inverse passes (Y, X, Z) in fp64 and certifies every
// pixel against Java's InverseDCT fold with |v_gpu - v_java| <= dec_G * L1 + dec_E (dct3d_plan.cpp).  The
// alternative: the first passes in fp32 (the encode's scheme), the last in fp64 (the fixed-point byte
// trick needs it).  This tool derives that variant's rigorous bound with the planner's own Tracked
// analysis of the same butterfly source (pass by pass unit roundoff and constant rounding), emulates its
// arithmetic on real cubes (dct_butterfly.h with T = float for the fp32 passes), and counts the pixels
// the certificate leaves open (they would go to a per-pixel fp64 re-evaluation or the exact fold).
//   g++ -O2 -std=c++17 -ffp-contract=off -shared -fPIC -I 3ddctvideoencoding_amd/csrc -I include \
//       tools/dec_f32_study.cpp -o /tmp/libdecf32.so      (tools/dec_f32_study.py drives it)
#include "dct3d_plan.cpp"

#include <cstdio>

using namespace dct3d;

namespace {

// per-pass arithmetic: 0 = fp64, 1 = fp32 (unit roundoff, constant rounding)
struct Mode {
    int y, x, z;
};

// the planner's analyse_decoder with a unit roundoff per pass; G = max_{n,i} ev + J |w| over all inputs,
// Gac = the same over the inputs i != 0 (the DC coefficient excluded)
void bound(int D, Mode m, double& G, double& Gac) {
    const int cs = 64 * D;
    const double J = (cs + 16) * std::ldexp(1.0, -52);
    g_ev = true;
    std::vector<Tracked> v(cs);
    for (int n = 0; n < cs; n++) {
        v[n] = Tracked(cs);
        v[n].w[n] = 1.0;
        v[n].ev.assign(cs, 0.0);
    }
    auto at = [&](int z, int y, int x) -> Tracked& { return v[(z * 8 + y) * 8 + x]; };
    auto set = [](int f32) {
        g_u = std::ldexp(1.0, f32 ? -24 : -53);
        g_f32 = f32 != 0;
    };
    set(m.y);
    for (int z = 0; z < D; z++)
        for (int x = 0; x < 8; x++) {
            Tracked r[8];
            for (int y = 0; y < 8; y++) r[y] = at(z, y, x);
            idct8(r);
            for (int y = 0; y < 8; y++) at(z, y, x) = r[y];
        }
    set(m.x);
    for (int z = 0; z < D; z++)
        for (int y = 0; y < 8; y++) {
            Tracked r[8];
            for (int x = 0; x < 8; x++) r[x] = at(z, y, x);
            idct8(r);
            for (int x = 0; x < 8; x++) at(z, y, x) = r[x];
        }
    set(m.z);
    for (int y = 0; y < 8; y++)
        for (int x = 0; x < 8; x++) {
            if (D == 8) {
                Tracked r[8];
                for (int z = 0; z < 8; z++) r[z] = at(z, y, x);
                idct8_fix(r, 0.0);
                for (int z = 0; z < 8; z++) at(z, y, x) = r[z];
            } else {
                Tracked r[4];
                for (int z = 0; z < 4; z++) r[z] = at(z, y, x);
                idct4_fix(r, 0.0);
                for (int z = 0; z < 4; z++) at(z, y, x) = r[z];
            }
        }
    g_ev = false;
    G = Gac = 0.0;
    for (int n = 0; n < cs; n++)
        for (int i = 0; i < cs; i++) {
            const double g = v[n].ev[i] + J * std::fabs(v[n].w[i]);
            G = std::max(G, g);
            if (i) Gac = std::max(Gac, g);
        }
}

template <class TY, class TX>
void emulate_cube(const int32_t* q, int D, double* out, double& l1, double& l1ac) {
    TY by[8][8][8];
    l1 = l1ac = 0.0;
    for (int z = 0; z < D; z++)
        for (int y = 0; y < 8; y++)
            for (int x = 0; x < 8; x++) {
                const double v = (double)q[(z * 8 + y) * 8 + x] * (double)std::max(1, 5 * (x + y + z));
                by[z][y][x] = (TY)v;  // exact in fp32 while |q step| < 2^24
                l1 += std::fabs(v);
                if (x | y | z) l1ac += std::fabs(v);
            }
    for (int z = 0; z < D; z++)
        for (int x = 0; x < 8; x++) {
            TY r[8];
            for (int y = 0; y < 8; y++) r[y] = by[z][y][x];
            idct8(r);
            for (int y = 0; y < 8; y++) by[z][y][x] = r[y];
        }
    TX bx[8][8][8];
    for (int z = 0; z < D; z++)
        for (int y = 0; y < 8; y++) {
            TX r[8];
            for (int x = 0; x < 8; x++) r[x] = (TX)by[z][y][x];
            idct8(r);
            for (int x = 0; x < 8; x++) bx[z][y][x] = r[x];
        }
    for (int y = 0; y < 8; y++)
        for (int x = 0; x < 8; x++) {
            if (D == 8) {
                double r[8];
                for (int z = 0; z < 8; z++) r[z] = (double)bx[z][y][x];
                idct8_fix(r, 0.0);
                for (int z = 0; z < 8; z++) out[(z * 8 + y) * 8 + x] = r[z];
            } else {
                double r[4];
                for (int z = 0; z < 4; z++) r[z] = (double)bx[z][y][x];
                idct4_fix(r, 0.0);
                for (int z = 0; z < 4; z++) out[(z * 8 + y) * 8 + x] = r[z];
            }
        }
}

}  // namespace

extern "C" {

// bounds of the three variants: out[0..5] = G, Gac for (fp64 all), (Y fp32), (Y, X fp32)
int study_bounds(int D, double* out) {
    const Mode modes[3] = {{0, 0, 0}, {1, 0, 0}, {1, 1, 0}};
    for (int i = 0; i < 3; i++) bound(D, modes[i], out[2 * i], out[2 * i + 1]);
    return 0;
}

// pixel values of n cubes under variant `mode` (0 fp64, 1 Y fp32, 2 Y and X fp32), plus each cube's L1
// and L1 without the DC term
int study_emulate(const int32_t* q, int n, int D, int mode, double* out, double* l1, double* l1ac) {
    const int cs = 64 * D;
    for (int g = 0; g < n; g++) {
        const int32_t* qc = q + (size_t)g * cs;
        double* o = out + (size_t)g * cs;
        if (mode == 0) emulate_cube<double, double>(qc, D, o, l1[g], l1ac[g]);
        else if (mode == 1) emulate_cube<float, double>(qc, D, o, l1[g], l1ac[g]);
        else emulate_cube<float, float>(qc, D, o, l1[g], l1ac[g]);
    }
    return 0;
}
}
