// dct_butterfly.h -- 8- and 4-point orthonormal DCT-II / DCT-III butterflies.
//
// ONE source for two consumers:
//   * the HIP kernels instantiate them with T = float / double;
//   * the host planner (dct3d_plan.cpp) instantiates them with T = Tracked, an abstract value that
//     carries the exact linear functional and a rigorous rounding-error bound, so the certification
//     bounds used by the fused encode kernel are derived from exactly the operation sequence the
//     kernel executes (compiled with -ffp-contract=off, so no op is fused behind our back).
//
// Maths: the reference Java transform (dct/DCT.java:77-112) computes, per 8x8x8 cube,
//   X[k0,k1,k2] = sqrt(8)/sqrt(cubeSize) * c(k0) c(k1) c(k2) * sum_n x[n] * prod cos(pi/N (n+1/2) k)
// with c(0) = 1/sqrt(2), which is exactly the separable orthonormal DCT-II along each axis
// (alpha_0 = sqrt(1/N), alpha_k = sqrt(2/N)); the 8x8x4 variant likewise.  The inverse
// (dct/InverseDCT.java:87-133) is the transpose.
//
// 8-point forward (36 ops: 8 add, 4 add, 2 add + 2 mul, 2 mul + 2 fma, 4 mul + 12 fma):
//   s_i = x_i + x_{7-i}, d_i = x_i - x_{7-i}                     (i = 0..3)
//   e0 = s0+s3, e1 = s1+s2, f0 = s0-s3, f1 = s1-s2
//   X0 = (e0+e1)*C4, X4 = (e0-e1)*C4,  X2 = A f0 + B f1,  X6 = B f0 - A f1
//   X_{2r+1} = sum_i M[r][i] d_i,  M[r][i] = cos((2i+1)(2r+1) pi/16)/2
#pragma once

#if defined(__HIPCC__) || defined(__HIP__)
#include <hip/hip_runtime.h>
#define DCT_HD __host__ __device__ __forceinline__
#else
#define DCT_HD inline
#endif

namespace dct3d {

// ---- exact constants (double); each consumer rounds them to its own T -----------------------
constexpr double kC4 = 0.35355339059327376220042218105242;   // 1/sqrt(8)
constexpr double kA8 = 0.46193976625564337806409159469839;   // cos(pi/8)/2
constexpr double kB8 = 0.19134171618254488586422999201520;   // cos(3pi/8)/2
constexpr double kC1 = 0.49039264020161522456309111806712;   // cos(pi/16)/2
constexpr double kC3 = 0.41573480615127261853939418880895;   // cos(3pi/16)/2
constexpr double kC5 = 0.27778511650980111237141540697427;   // cos(5pi/16)/2
constexpr double kC7 = 0.09754516100806413392146691110355;   // cos(7pi/16)/2
constexpr double kP4 = 0.65328148243818826392832158671359;   // cos(pi/8)/sqrt(2)
constexpr double kQ4 = 0.27059805007309849219986160268319;   // cos(3pi/8)/sqrt(2)

// ---- primitive ops: default (float/double) implementations --------------------------------
// EX = the operation is known to be exact (integer-valued operands in pass X of the encoder);
// the device ignores it, the Tracked analysis skips the rounding term.
template <bool EX = false, class T> DCT_HD T dadd(const T& a, const T& b) { return a + b; }
template <bool EX = false, class T> DCT_HD T dsub(const T& a, const T& b) { return a - b; }
template <class T> DCT_HD T dmulc(double c, const T& a) { return T(c) * a; }
template <class T> DCT_HD T dfmac(double c, const T& a, const T& b);  // c*a + b, one rounding
template <> DCT_HD float dfmac<float>(double c, const float& a, const float& b) {
    return __builtin_fmaf(float(c), a, b);
}
template <> DCT_HD double dfmac<double>(double c, const double& a, const double& b) {
    return __builtin_fma(c, a, b);
}
// multiplication by an exact power of two (0.5): exact in floating point
template <class T> DCT_HD T dhalf(const T& a) { return T(0.5) * a; }
// negation: exact
template <class T> DCT_HD T dneg(const T& a) { return -a; }
// c*a + K and a/2 + K, one rounding (the decode's fixed-point offset; Tracked: c*a and a/2)
template <class T> DCT_HD T dfmac_k(double c, const T& a, double K) { return dfmac(c, a, T(K)); }
template <class T> DCT_HD T dhalf_k(const T& a, double K) { return dfmac(0.5, a, T(K)); }

// ---- 8-point forward DCT-II (orthonormal), in place ---------------------------------------
// dcsub: subtracted from (e0 + e1) before scaling (the encoder folds its cube-mean centring in
// here: sum_i (x_i - m) = e0 + e1 - 8m, exact in integers).  EXF: the front (adds) are exact.
template <bool EXF, bool HAS_DCSUB, class T>
DCT_HD void fdct8(T (&x)[8], const T& dcsub) {
    T s0 = dadd<EXF>(x[0], x[7]), s1 = dadd<EXF>(x[1], x[6]);
    T s2 = dadd<EXF>(x[2], x[5]), s3 = dadd<EXF>(x[3], x[4]);
    T d0 = dsub<EXF>(x[0], x[7]), d1 = dsub<EXF>(x[1], x[6]);
    T d2 = dsub<EXF>(x[2], x[5]), d3 = dsub<EXF>(x[3], x[4]);
    T e0 = dadd<EXF>(s0, s3), e1 = dadd<EXF>(s1, s2);
    T f0 = dsub<EXF>(s0, s3), f1 = dsub<EXF>(s1, s2);
    T ee = dadd<EXF>(e0, e1);
    if constexpr (HAS_DCSUB) ee = dsub<EXF>(ee, dcsub);
    x[0] = dmulc(kC4, ee);
    x[4] = dmulc(kC4, dsub<EXF>(e0, e1));
    x[2] = dfmac(kB8, f1, dmulc(kA8, f0));
    x[6] = dfmac(-kA8, f1, dmulc(kB8, f0));
    x[1] = dfmac(kC7, d3, dfmac(kC5, d2, dfmac(kC3, d1, dmulc(kC1, d0))));
    x[3] = dfmac(-kC5, d3, dfmac(-kC1, d2, dfmac(-kC7, d1, dmulc(kC3, d0))));
    x[5] = dfmac(kC3, d3, dfmac(kC7, d2, dfmac(-kC1, d1, dmulc(kC5, d0))));
    x[7] = dfmac(-kC1, d3, dfmac(kC3, d2, dfmac(-kC5, d1, dmulc(kC7, d0))));
}

// ---- 4-point forward DCT-II (orthonormal) ---------------------------------------------------
//   s0=x0+x3, s1=x1+x2, d0=x0-x3, d1=x1-x2
//   X0=(s0+s1)/2, X2=(s0-s1)/2, X1=P d0 + Q d1, X3 = Q d0 - P d1   (P,Q = cos(pi/8),cos(3pi/8) / sqrt2)
template <bool EXF, bool HAS_DCSUB, class T>
DCT_HD void fdct4(T (&x)[4], const T& dcsub) {
    T s0 = dadd<EXF>(x[0], x[3]), s1 = dadd<EXF>(x[1], x[2]);
    T d0 = dsub<EXF>(x[0], x[3]), d1 = dsub<EXF>(x[1], x[2]);
    T ss = dadd<EXF>(s0, s1);
    if constexpr (HAS_DCSUB) ss = dsub<EXF>(ss, dcsub);
    x[0] = dhalf(ss);
    x[2] = dhalf(dsub<EXF>(s0, s1));
    x[1] = dfmac(kQ4, d1, dmulc(kP4, d0));
    x[3] = dfmac(-kP4, d1, dmulc(kQ4, d0));
}

// ---- 8-point inverse (DCT-III, orthonormal) -------------------------------------------------
//   E0 = C4(X0+X4) + (A X2 + B X6), E3 = C4(X0+X4) - (A X2 + B X6)
//   E1 = C4(X0-X4) + (B X2 - A X6), E2 = C4(X0-X4) - (B X2 - A X6)
//   O_n = sum_r M[r][n] X_{2r+1};  x_n = E_n + O_n, x_{7-n} = E_n - O_n
// idct8: the C4 scale fused into the even combine (E = fma(C4, X0 +- X4, +-r)): 34 ops.
// idct8_fix: the decode's last pass: p = fma(C4, X0 + X4, K), q = fma(C4, X0 - X4, K) put the
// fixed-point offset K into every output at no cost (36 ops).  For the Tracked analysis dfmac_k is the
// plain product C4 * s (K = 0); the offset form's three roundings in [2^20, 2^21) (p, E, x: <= 2^-33
// each, instead of the relative roundings the analysis counts) are added by the planner (dec_E).
template <class T>
DCT_HD void idct8(T (&X)[8]) {
    const T s = dadd(X[0], X[4]), d = dsub(X[0], X[4]);
    const T r0 = dfmac(kB8, X[6], dmulc(kA8, X[2]));
    const T r1 = dfmac(-kA8, X[6], dmulc(kB8, X[2]));
    const T E0 = dfmac(kC4, s, r0), E3 = dfmac(kC4, s, dneg(r0));
    const T E1 = dfmac(kC4, d, r1), E2 = dfmac(kC4, d, dneg(r1));
    T O0 = dfmac(kC7, X[7], dfmac(kC5, X[5], dfmac(kC3, X[3], dmulc(kC1, X[1]))));
    T O1 = dfmac(-kC5, X[7], dfmac(-kC1, X[5], dfmac(-kC7, X[3], dmulc(kC3, X[1]))));
    T O2 = dfmac(kC3, X[7], dfmac(kC7, X[5], dfmac(-kC1, X[3], dmulc(kC5, X[1]))));
    T O3 = dfmac(-kC1, X[7], dfmac(kC3, X[5], dfmac(-kC5, X[3], dmulc(kC7, X[1]))));
    X[0] = dadd(E0, O0); X[7] = dsub(E0, O0);
    X[1] = dadd(E1, O1); X[6] = dsub(E1, O1);
    X[2] = dadd(E2, O2); X[5] = dsub(E2, O2);
    X[3] = dadd(E3, O3); X[4] = dsub(E3, O3);
}
template <class T>
DCT_HD void idct8_fix(T (&X)[8], double K) {
    const T p = dfmac_k(kC4, dadd(X[0], X[4]), K);
    const T q = dfmac_k(kC4, dsub(X[0], X[4]), K);
    const T r0 = dfmac(kB8, X[6], dmulc(kA8, X[2]));
    const T r1 = dfmac(-kA8, X[6], dmulc(kB8, X[2]));
    const T E0 = dadd(p, r0), E3 = dsub(p, r0), E1 = dadd(q, r1), E2 = dsub(q, r1);
    T O0 = dfmac(kC7, X[7], dfmac(kC5, X[5], dfmac(kC3, X[3], dmulc(kC1, X[1]))));
    T O1 = dfmac(-kC5, X[7], dfmac(-kC1, X[5], dfmac(-kC7, X[3], dmulc(kC3, X[1]))));
    T O2 = dfmac(kC3, X[7], dfmac(kC7, X[5], dfmac(-kC1, X[3], dmulc(kC5, X[1]))));
    T O3 = dfmac(-kC1, X[7], dfmac(kC3, X[5], dfmac(-kC5, X[3], dmulc(kC7, X[1]))));
    X[0] = dadd(E0, O0); X[7] = dsub(E0, O0);
    X[1] = dadd(E1, O1); X[6] = dsub(E1, O1);
    X[2] = dadd(E2, O2); X[5] = dsub(E2, O2);
    X[3] = dadd(E3, O3); X[4] = dsub(E3, O3);
}

// ---- 4-point inverse --------------------------------------------------------------------------
//   E0 = (X0+X2)/2, E1 = (X0-X2)/2, O0 = P X1 + Q X3, O1 = Q X1 - P X3
template <class T>
DCT_HD void idct4(T (&X)[4]) {
    T E0 = dhalf(dadd(X[0], X[2])), E1 = dhalf(dsub(X[0], X[2]));
    T O0 = dfmac(kQ4, X[3], dmulc(kP4, X[1]));
    T O1 = dfmac(-kP4, X[3], dmulc(kQ4, X[1]));
    X[0] = dadd(E0, O0); X[3] = dsub(E0, O0);
    X[1] = dadd(E1, O1); X[2] = dsub(E1, O1);
}
// the decode's last pass at depth 4: E = fma(1/2, X0 +- X2, K) (Tracked: the exact halving; the offset
// form's two roundings in [2^20, 2^21) are covered by the planner's dec_E as for idct8_fix)
template <class T>
DCT_HD void idct4_fix(T (&X)[4], double K) {
    T E0 = dhalf_k(dadd(X[0], X[2]), K), E1 = dhalf_k(dsub(X[0], X[2]), K);
    T O0 = dfmac(kQ4, X[3], dmulc(kP4, X[1]));
    T O1 = dfmac(-kP4, X[3], dmulc(kQ4, X[1]));
    X[0] = dadd(E0, O0); X[3] = dsub(E0, O0);
    X[1] = dadd(E1, O1); X[2] = dsub(E1, O1);
}

// depth-generic forward / inverse along one axis
template <int N, bool EXF, bool HAS_DCSUB, class T>
DCT_HD void fdctN(T (&x)[N], const T& dcsub) {
    if constexpr (N == 8) fdct8<EXF, HAS_DCSUB>(x, dcsub);
    else fdct4<EXF, HAS_DCSUB>(x, dcsub);
}
template <int N, class T>
DCT_HD void idctN(T (&x)[N]) {
    if constexpr (N == 8) idct8(x);
    else idct4(x);
}
template <int N, class T>
DCT_HD void idctN_fix(T (&x)[N], double K) {
    if constexpr (N == 8) idct8_fix(x, K);
    else idct4_fix(x, K);
}

}  // namespace dct3d
