// dct3d_plan.cpp -- transform plan + certification bounds (host side, built into libdct3d.so).
//
// 1. Java grouping (DCT.java:77-140): for every output coefficient k the reference computes the
//    coefficients of all 512 inputs, keys them by (long)(c * 1e9) in a java.util.HashMap<Long,..>
//    (first inserted member's coefficient wins), drops key == 0, and folds
//        out[k] = (((0 + S_g0*c_g0) + S_g1*c_g1) + ...)       (DCT.java:49-55, Sum.java:41-52)
//    in HashMap iteration order (DCT.java:98).  S_g are sums of integer pixels, exact in double, so
//    the Java result is fully determined by (group membership, group coefficient bits, fold order).
//    This file re-derives all three with a Java 8 HashMap emulation; the device exact-fold path
//    (the kernels' in-wave replays) repeats that fold bit for bit.
// 2. Certification bounds: the fp32 fused encoder is analysed by running the kernel's own
//    butterflies (dct_butterfly.h) on a Tracked value type that carries the exact linear functional
//    and a rigorous rounding-error bound.  Any coefficient whose fp32 quotient lies within the bound
//    of a rounding tie is re-done by the exact fold, so the quantised output equals the Java fold
//    bit for bit.
#include "dct3d_plan.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

namespace dct3d {

// =============================================================================================
// Tracked value (error analysis)
// =============================================================================================
struct Tracked {
    std::vector<double> w;   // exact linear functional over the cube's inputs
    double e = 0.0;          // rounding-error bound for inputs with |x_n| <= 1
    std::vector<double> ev;  // (decoder analysis) per-input error coefficients: error <= sum_n ev[n] |x_n|
    Tracked() = default;
    explicit Tracked(size_t n) : w(n, 0.0) {}
};

namespace {
double g_u = 0.0;     // unit roundoff of the analysed arithmetic
bool g_f32 = true;    // constants rounded to float (else double)
bool g_ev = false;    // track the per-input error coefficients (Tracked::ev)
double l1(const std::vector<double>& w) {
    double s = 0;
    for (double x : w) s += std::fabs(x);
    return s;
}
double crep(double c) { return g_f32 ? (double)(float)c : c; }
// |stored constant - true constant|: rounding to T plus the double literal's own error
double cerr(double c) { return std::fabs(crep(c) - c) + std::ldexp(std::fabs(c), -53); }
// one rounding of the result: |rounded - exact| <= u |exact| <= u (sum |w_n x_n| + error), i.e. per
// input n: u (|w_n| + ev_n)
void round_term(Tracked& r, bool exact) {
    if (exact) return;
    r.e += g_u * (l1(r.w) + r.e);
    for (size_t i = 0; i < r.ev.size(); i++) r.ev[i] += g_u * (std::fabs(r.w[i]) + r.ev[i]);
}
Tracked make_like(const Tracked& a) {
    Tracked r(a.w.size());
    if (g_ev) r.ev.assign(a.w.size(), 0.0);
    return r;
}
}  // namespace

template <bool EX = false>
inline Tracked dadd(const Tracked& a, const Tracked& b) {
    Tracked r = make_like(a);
    for (size_t i = 0; i < r.w.size(); i++) r.w[i] = a.w[i] + b.w[i];
    for (size_t i = 0; i < r.ev.size(); i++) r.ev[i] = a.ev[i] + b.ev[i];
    r.e = a.e + b.e;
    round_term(r, EX);
    return r;
}
template <bool EX = false>
inline Tracked dsub(const Tracked& a, const Tracked& b) {
    Tracked r = make_like(a);
    for (size_t i = 0; i < r.w.size(); i++) r.w[i] = a.w[i] - b.w[i];
    for (size_t i = 0; i < r.ev.size(); i++) r.ev[i] = a.ev[i] + b.ev[i];
    r.e = a.e + b.e;
    round_term(r, EX);
    return r;
}
inline Tracked dmulc(double c, const Tracked& a) {
    Tracked r = make_like(a);
    for (size_t i = 0; i < r.w.size(); i++) r.w[i] = c * a.w[i];
    for (size_t i = 0; i < r.ev.size(); i++) r.ev[i] = std::fabs(crep(c)) * a.ev[i] + cerr(c) * std::fabs(a.w[i]);
    r.e = std::fabs(crep(c)) * a.e + cerr(c) * l1(a.w);
    round_term(r, false);
    return r;
}
inline Tracked dfmac(double c, const Tracked& a, const Tracked& b) {
    Tracked r = make_like(a);
    for (size_t i = 0; i < r.w.size(); i++) r.w[i] = c * a.w[i] + b.w[i];
    for (size_t i = 0; i < r.ev.size(); i++)
        r.ev[i] = std::fabs(crep(c)) * a.ev[i] + cerr(c) * std::fabs(a.w[i]) + b.ev[i];
    r.e = std::fabs(crep(c)) * a.e + cerr(c) * l1(a.w) + b.e;
    round_term(r, false);
    return r;
}
inline Tracked dneg(const Tracked& a) {
    Tracked r = a;
    for (double& x : r.w) x = -x;
    return r;
}
// the decode's offset forms: analysed as the plain product / halving (see dct_butterfly.h idct8_fix)
inline Tracked dfmac_k(double c, const Tracked& a, double) { return dmulc(c, a); }
inline Tracked dhalf(const Tracked& a) {
    Tracked r = make_like(a);
    for (size_t i = 0; i < r.w.size(); i++) r.w[i] = 0.5 * a.w[i];
    for (size_t i = 0; i < r.ev.size(); i++) r.ev[i] = 0.5 * a.ev[i];
    r.e = 0.5 * a.e;
    return r;
}
inline Tracked dhalf_k(const Tracked& a, double) { return dhalf(a); }

}  // namespace dct3d

#include "dct_butterfly.h"

namespace dct3d {

// =============================================================================================
// Java 8 java.util.HashMap<Long, V> emulation (insertion + iteration order)
// =============================================================================================
namespace {

struct JavaLongMap {
    struct Node {
        uint32_t hash;
        int64_t key;
        int val;
        int next;
    };
    std::vector<int> table;  // bin heads
    std::vector<Node> nodes;
    int size = 0, threshold = 0;
    bool treeified = false;

    static uint32_t spread(int64_t key) {
        uint64_t v = (uint64_t)key;
        uint32_t h = (uint32_t)(v ^ (v >> 32));  // Long.hashCode
        return h ^ (h >> 16);                    // HashMap.hash
    }
    void resize() {
        if (table.empty()) {
            table.assign(16, -1);
            threshold = 12;
            return;
        }
        const int oldCap = (int)table.size();
        std::vector<int> nt(2 * oldCap, -1);
        for (int j = 0; j < oldCap; j++) {
            int loH = -1, loT = -1, hiH = -1, hiT = -1;
            for (int e = table[j]; e >= 0;) {
                int nx = nodes[e].next;
                nodes[e].next = -1;
                if ((nodes[e].hash & (uint32_t)oldCap) == 0) {
                    (loT < 0 ? loH : nodes[loT].next) = e;
                    loT = e;
                } else {
                    (hiT < 0 ? hiH : nodes[hiT].next) = e;
                    hiT = e;
                }
                e = nx;
            }
            nt[j] = loH;
            nt[j + oldCap] = hiH;
        }
        table.swap(nt);
        threshold *= 2;
    }
    int get(int64_t key) const {
        if (table.empty()) return -1;
        uint32_t h = spread(key);
        for (int e = table[h & (table.size() - 1)]; e >= 0; e = nodes[e].next)
            if (nodes[e].key == key) return nodes[e].val;
        return -1;
    }
    void put_absent(int64_t key, int val) {  // HashMap.putVal for a key known to be absent
        if (table.empty()) resize();
        uint32_t h = spread(key);
        int id = (int)nodes.size();
        nodes.push_back({h, key, val, -1});
        size_t i = h & (table.size() - 1);
        if (table[i] < 0) {
            table[i] = id;
        } else {
            int p = table[i], binCount = 0;
            while (nodes[p].next >= 0) {
                p = nodes[p].next;
                binCount++;
            }
            nodes[p].next = id;
            if (binCount >= 7) {                        // TREEIFY_THRESHOLD - 1
                if (table.size() < 64) resize();        // MIN_TREEIFY_CAPACITY
                else treeified = true;
            }
        }
        if (++size > threshold) resize();
    }
    template <class F>
    void for_each_value(F f) const {
        for (int head : table)
            for (int e = head; e >= 0; e = nodes[e].next) f(nodes[e].val);
    }
};

int64_t java_d2l(double d) {
    if (d != d) return 0;
    if (d >= 9223372036854775807.0) return INT64_MAX;
    if (d <= -9223372036854775808.0) return INT64_MIN;
    return (int64_t)d;
}

// DCT.java:100-110 / InverseDCT.java:108-123, evaluated strictly left to right like javac.
double java_coefficient(int cw, int ch, int cd, int k0, int k1, int k2, int n0, int n1, int n2) {
    const double DIMENSIONAL_FACTOR = std::sqrt(std::pow(2.0, 3.0));  // Transform.java:20
    const double INVERSE_SQRT_2 = 1.0 / std::sqrt(2.0);             // Transform.java:21
    const volatile double scale = DIMENSIONAL_FACTOR / std::sqrt((double)(cw * ch * cd));
    const double piOverWidth = M_PI / (double)(float)cw;
    const double piOverHeight = M_PI / (double)(float)ch;
    const double piOverDepth = M_PI / (double)(float)cd;
    double c0 = k0 == 0 ? INVERSE_SQRT_2 : 1.0;
    double c1 = k1 == 0 ? INVERSE_SQRT_2 : 1.0;
    double c2 = k2 == 0 ? INVERSE_SQRT_2 : 1.0;
    volatile double a0 = piOverDepth * (double)((float)n0 + 0.5f);
    a0 = a0 * (double)k0;
    volatile double a1 = piOverHeight * (double)((float)n1 + 0.5f);
    a1 = a1 * (double)k1;
    volatile double a2 = piOverWidth * (double)((float)n2 + 0.5f);
    a2 = a2 * (double)k2;
    volatile double c = scale * c0;
    c = c * c1;
    c = c * c2;
    c = c * std::cos((double)a0);
    c = c * std::cos((double)a1);
    c = c * std::cos((double)a2);
    return c;
}

}  // namespace

// =============================================================================================
// Error analysis of the fused kernels
// =============================================================================================
namespace {

// Encoder: kernel order = pass X (exact integer front, cube-mean centring) -> pass Z -> pass Y, fp32.
void analyse_encoder(Plan& p) {
    const int D = p.cd, cs = p.cs;
    g_u = std::ldexp(1.0, -24);
    g_f32 = true;
    std::vector<Tracked> v(cs);
    for (int n = 0; n < cs; n++) {
        v[n] = Tracked(cs);
        v[n].w[n] = 1.0;
    }
    auto at = [&](int z, int y, int x) -> Tracked& { return v[(z * 8 + y) * 8 + x]; };
    Tracked zero(cs);
    for (int z = 0; z < D; z++)
        for (int y = 0; y < 8; y++) {
            Tracked r[8];
            for (int x = 0; x < 8; x++) r[x] = at(z, y, x);
            fdct8<true, true>(r, zero);
            for (int x = 0; x < 8; x++) at(z, y, x) = r[x];
        }
    for (int y = 0; y < 8; y++)
        for (int x = 0; x < 8; x++) {
            if (D == 8) {
                Tracked r[8];
                for (int z = 0; z < 8; z++) r[z] = at(z, y, x);
                fdct8<false, false>(r, zero);
                for (int z = 0; z < 8; z++) at(z, y, x) = r[z];
            } else {
                Tracked r[4];
                for (int z = 0; z < 4; z++) r[z] = at(z, y, x);
                fdct4<false, false>(r, zero);
                for (int z = 0; z < 4; z++) at(z, y, x) = r[z];
            }
        }
    for (int z = 0; z < D; z++)
        for (int x = 0; x < 8; x++) {
            Tracked r[8];
            for (int y = 0; y < 8; y++) r[y] = at(z, y, x);
            fdct8<false, false>(r, zero);
            for (int y = 0; y < 8; y++) at(z, y, x) = r[y];
        }
    p.enc_K.assign(cs, 0.0);
    p.enc_L1.assign(cs, 0.0);
    for (int k = 0; k < cs; k++) {
        p.enc_K[k] = v[k].e;
        p.enc_L1[k] = l1(v[k].w);
    }
}

// Decoder: kernel order = inverse pass Y (face layout) -> inverse pass X -> inverse pass Z, fp64.
// Returns, per output n: K[n] = error bound for unit inputs (sum_i ev[n][i]), L1[n] = sum_i |w[n][i]|,
// and G1 = max over n, i of ev[n][i] + J |w[n][i]| (J: the Java fold's own error per unit term), the
// error per unit of sum_i |x_i|; Bmax = max |w[n][i]| (|v_n| <= Bmax sum_i |x_i|).
void analyse_decoder(Plan& p, std::vector<double>& K, std::vector<double>& L1, double J, double& G1, double& Bmax) {
    const int D = p.cd, cs = p.cs;
    g_u = std::ldexp(1.0, -53);
    g_f32 = false;
    g_ev = true;
    std::vector<Tracked> v(cs);
    for (int n = 0; n < cs; n++) {
        v[n] = Tracked(cs);
        v[n].w[n] = 1.0;
        v[n].ev.assign(cs, 0.0);
    }
    auto at = [&](int z, int y, int x) -> Tracked& { return v[(z * 8 + y) * 8 + x]; };
    for (int z = 0; z < D; z++)
        for (int x = 0; x < 8; x++) {
            Tracked r[8];
            for (int y = 0; y < 8; y++) r[y] = at(z, y, x);
            idct8(r);
            for (int y = 0; y < 8; y++) at(z, y, x) = r[y];
        }
    for (int z = 0; z < D; z++)
        for (int y = 0; y < 8; y++) {
            Tracked r[8];
            for (int x = 0; x < 8; x++) r[x] = at(z, y, x);
            idct8(r);
            for (int x = 0; x < 8; x++) at(z, y, x) = r[x];
        }
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
    K.assign(cs, 0.0);
    L1.assign(cs, 0.0);
    G1 = 0.0;
    Bmax = 0.0;
    for (int n = 0; n < cs; n++) {
        K[n] = v[n].e;
        L1[n] = l1(v[n].w);
        for (int i = 0; i < cs; i++) {
            G1 = std::max(G1, v[n].ev[i] + J * std::fabs(v[n].w[i]));
            Bmax = std::max(Bmax, std::fabs(v[n].w[i]));
        }
    }
}

}  // namespace

// =============================================================================================
// Plan construction
// =============================================================================================
bool build_plan(int cw, int ch, int cd, Plan& p) {
    if (cw != 8 || ch != 8 || (cd != 8 && cd != 4)) return false;
    p = Plan();
    p.cw = cw;
    p.ch = ch;
    p.cd = cd;
    const int cs = cw * ch * cd;
    p.cs = cs;
    p.fwd_ngroups.assign(cs, 0);
    p.fwd_coef.assign((size_t)cs * kMaxGroups, 0.0);
    p.fwd_group_of.assign((size_t)cs * cs, 0xFF);
    p.enc_dev.assign(cs, 0.0);

    // ---- forward grouping (DCT.initialize) ----
    std::vector<double> own(cs);
    for (int k0 = 0, k = 0; k0 < cd; k0++)
        for (int k1 = 0; k1 < ch; k1++)
            for (int k2 = 0; k2 < cw; k2++, k++) {
                JavaLongMap map;
                std::vector<double> gcoef;
                std::vector<std::vector<int>> gmem;
                for (int n0 = 0; n0 < cd; n0++)
                    for (int n1 = 0; n1 < ch; n1++)
                        for (int n2 = 0; n2 < cw; n2++) {
                            const int n = (n0 * ch + n1) * cw + n2;
                            double c = java_coefficient(cw, ch, cd, k0, k1, k2, n0, n1, n2);
                            own[n] = c;
                            int64_t key = java_d2l(c * 1E9);
                            if (key == 0) continue;  // DCT.java:84 drops zero keys
                            int g = map.get(key);
                            if (g < 0) {
                                g = (int)gcoef.size();
                                gcoef.push_back(c);
                                gmem.emplace_back();
                                map.put_absent(key, g);
                            }
                            gmem[g].push_back(n);
                        }
                if (map.treeified) p.treeified = true;
                int order = 0;
                double dev = 0.0;
                bool overflow = false;
                map.for_each_value([&](int g) {
                    if (order >= kMaxGroups) {
                        overflow = true;
                        return;
                    }
                    p.fwd_coef[(size_t)k * kMaxGroups + order] = gcoef[g];
                    for (int n : gmem[g]) {
                        p.fwd_group_of[(size_t)k * cs + n] = (uint8_t)order;
                        dev += std::fabs(gcoef[g] - own[n]);
                    }
                    order++;
                });
                if (overflow) return false;
                p.fwd_ngroups[k] = order;
                p.n_mults += order;
                p.enc_dev[k] = dev;
                // dropped inputs (key == 0) contribute |own[n]| * 255 to the deviation
                for (int n = 0; n < cs; n++)
                    if (p.fwd_group_of[(size_t)k * cs + n] == 0xFF) p.enc_dev[k] += std::fabs(own[n]);
            }
    if (p.fwd_ngroups[0] != 1) return false;  // the kernels take the DC as one exact product
    if (cd == 4)  // the 8x8x4 encode's in-wave fold keeps kMaxGroups4 sums per cube (40 needed)
        for (int k = 0; k < cs; k++)
            if (p.fwd_ngroups[k] > kMaxGroups4) return false;
    p.coef_dc = p.fwd_coef[0];

    // ---- inverse coefficient matrix (InverseDCT.initialize) ----
    p.inv_coef.assign((size_t)cs * cs, 0.0);
    for (int n0 = 0; n0 < cd; n0++)
        for (int n1 = 0; n1 < ch; n1++)
            for (int n2 = 0; n2 < cw; n2++) {
                const int n = (n0 * ch + n1) * cw + n2;
                for (int k0 = 0; k0 < cd; k0++)
                    for (int k1 = 0; k1 < ch; k1++)
                        for (int k2 = 0; k2 < cw; k2++) {
                            const int k = (k0 * ch + k1) * cw + k2;
                            p.inv_coef[(size_t)n * cs + k] = java_coefficient(cw, ch, cd, k0, k1, k2, n0, n1, n2);
                        }
            }

    // ---- encoder certification tables ----
    analyse_encoder(p);
    const double u32 = std::ldexp(1.0, -24);
    double G[kMaxS] = {}, E[kMaxS] = {};
    for (int kz = 0; kz < cd; kz++)
        for (int ky = 0; ky < 8; ky++)
            for (int kx = 0; kx < 8; kx++) {
                const int k = (kz * 8 + ky) * 8 + kx;
                const int s = kx + ky + kz;
                if (s == 0) continue;  // DC is produced exactly from the integer cube sum
                const double step = std::max(1, 5 * s);
                const double K = p.enc_K[k], L1 = p.enc_L1[k];
                // |q_f - q_java| <= A*[K + 2.02u(L1+K) + 2^-50 L1]/step
                //                   + [255*dev + (ng+16) 2^-52 255 L1]/step + 1e-12
                const double gk = (K + 2.02 * u32 * (L1 + K) + std::ldexp(L1, -50)) / step;
                const double ek = (255.0 * p.enc_dev[k] + (p.fwd_ngroups[k] + 16) * std::ldexp(255.0 * L1, -52)) / step + 1e-12;
                G[s] = std::max(G[s], gk);
                E[s] = std::max(E[s], ek);
            }
    for (int s = 0; s < kMaxS; s++) {
        const double step = std::max(1, 5 * s);
        p.enc_rstep[s] = (float)(1.0 / step);
        if (s == 0) {
            p.enc_G[s] = 0.0f;
            p.enc_E[s] = -INFINITY;  // threshold +inf: the DC is never flagged
            continue;
        }
        // round up (conservative) and guard the fp32 evaluation of 0.5 - (A*G + E) in the kernel
        p.enc_G[s] = std::nextafter((float)(G[s] * (1.0 + 1e-4)), INFINITY);
        p.enc_E[s] = std::nextafter((float)(E[s] + 2e-7), INFINITY);
    }

    // ---- second certificate (8x8x8): fp64 re-evaluation of a coefficient the fp32 one leaves open ----
    // The kernel (e16_recheck64) computes v64 = sum over its 16 lanes of
    //   b[ky][y] * sum_e b[kz][4h+e] * sum_x x * b[kx][x]     (fp64 fma chains, xor-butterfly sum)
    // with b = basis64 (each entry the double nearest the exact basis value).  Against the exact
    // value V = sum_n x_n c_n (c_n the exact orthonormal basis product, 0 <= x_n <= 255):
    //   |v64 - V|    <= 72 u * 255 * L1x          (3 representation + 8 fma + 2 mul + 2 fma + 4 add
    //                                              roundings, each <= u * sum |terms|; 72u leaves 3x)
    //   |v_java - V| <= 255 * devx + (ng + 2) u * 255 * L1j
    //        devx = sum_n |cj_n - c_n|, cj_n = Java's group coefficient of input n (0 if dropped:
    //        DCT.java:84), L1j = sum_n |cj_n| (the fold's ng products and additions, DCT.java:49-52)
    // Both quotients by the step round once more (|q| < 2^12: 2^-40 each).  So with
    //   E64 = (255 devx + (ng + 2) u 255 L1j + 72 u 255 L1x) / step + 2^-38,
    // |q64 - rint(q64)| < 0.5 - E64 implies Math.round(v_java / step) = rint(q64).  The table holds
    // 0.5 - 2 max_k E64 per s (a further factor 2).  Exact values: long double (64-bit mantissa).
    if (cd == 8) {
        const long double pi = 3.141592653589793238462643383279502884L;
        long double bl[8][8];
        for (int kk = 0; kk < 8; kk++)
            for (int n = 0; n < 8; n++) {
                bl[kk][n] = (kk == 0 ? sqrtl(0.125L) : 0.5L) * cosl(pi * (long double)((2 * n + 1) * kk) / 16.0L);
                p.basis64[kk * 8 + n] = (double)bl[kk][n];
            }
        const long double u = ldexpl(1.0L, -53);
        long double E64[kMaxS] = {};
        for (int kz = 0; kz < 8; kz++)
            for (int ky = 0; ky < 8; ky++)
                for (int kx = 0; kx < 8; kx++) {
                    const int k = (kz * 8 + ky) * 8 + kx, s = kx + ky + kz;
                    if (s == 0) continue;
                    long double devx = 0, L1x = 0, L1j = 0;
                    for (int z = 0; z < 8; z++)
                        for (int y = 0; y < 8; y++)
                            for (int x = 0; x < 8; x++) {
                                const int n = (z * 8 + y) * 8 + x;
                                const long double ex = bl[kz][z] * bl[ky][y] * bl[kx][x];
                                const uint8_t go = p.fwd_group_of[(size_t)k * cs + n];
                                const long double cj = go == 0xFF ? 0.0L : (long double)p.fwd_coef[(size_t)k * kMaxGroups + go];
                                devx += fabsl(cj - ex);
                                L1x += fabsl(ex);
                                L1j += fabsl(cj);
                            }
                    const long double e = (255.0L * devx + (p.fwd_ngroups[k] + 2) * u * 255.0L * L1j +
                                           72.0L * u * 255.0L * L1x) / (long double)(5 * s) +
                                          ldexpl(1.0L, -38);
                    E64[s] = std::max(E64[s], e);
                }
        for (int s = 0; s < kMaxS; s++) p.enc_thr64[s] = s == 0 ? 0.5 : (double)(0.5L - 2.0L * E64[s]);
    }

    // ---- decoder certification (fp64 kernel vs the Java fold) ----
    // Java's fold (InverseDCT.java:56-66) of at most cs products, each rounded, its coefficients within
    // a few ulps of the exact basis: |v_java - v_exact| <= J sum_k |x_k B_nk| with J = (cs + 16) 2^-52.
    // The kernel: |v_gpu - v_exact| <= sum_k ev[n][k] |x_k| (analyse_decoder).  So with
    // L1x = sum_k |x_k| (the kernel's upper bound of it), |v_gpu - v_java| <= G1 L1x (+ dec_E).
    std::vector<double> Kd, L1d;
    double G1 = 0.0, Bmax = 0.0;
    const double J = (cs + 16) * std::ldexp(1.0, -52);
    analyse_decoder(p, Kd, L1d, J, G1, Bmax);
    double gd = 0.0;
    for (int n = 0; n < cs; n++) gd = std::max(gd, Kd[n] + J * L1d[n]);
    p.dec_G = G1 * (1.0 + 1e-3);
    // + the last pass's offset form (idct8_fix / idct4_fix): at most three roundings of values in
    // [2^20, 2^21), 2^-33 each, beyond what the analysis counts
    p.dec_E = 1e-12 + 3.0 * std::ldexp(1.0, -33);
    // the kernel's byte packing reads floor(v) as a signed 16-bit value: |v| <= Bmax L1x must stay below
    // 2^15 - 1 (with room for the error terms)
    p.dec_l1_max = (float)(32000.0 / Bmax);
    p.fwd64_K = gd;
    return true;
}

}  // namespace dct3d
