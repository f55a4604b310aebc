// dct3d_plan.h -- host-side transform plan (the MI355X build's equivalent of DCT.initialize /
// InverseDCT.initialize, /root/reference/3d-DCT-video-encoding/src/br/jpiccoli/video/dct/
// DCT.java:77-163 and InverseDCT.java:87-133), plus the certification bounds of the fused kernels.
#pragma once
#include <cstdint>
#include <vector>

namespace dct3d {

constexpr int kMaxGroups = 64;   // per-coefficient group slots in the device fold table
constexpr int kMaxGroups4 = 48;  // 8x8x4: group sums per cube of the encode's in-wave fold (kGM4Dev)
constexpr int kMaxS = 32;        // s = kx + ky + kz table size (max 21 for 8x8x8)

struct Plan {
    int cw = 8, ch = 8, cd = 8, cs = 512;

    // ---- Java forward fold (DCT.java:77-112 + HashMap<Long,..> iteration order) ----
    std::vector<int32_t> fwd_ngroups;     // [cs]
    std::vector<double> fwd_coef;         // [cs * kMaxGroups], fold order
    std::vector<uint8_t> fwd_group_of;    // [cs * cs]  group (fold index) of input n for output k
    int n_mults = 0;                      // sum of fwd_ngroups (11,567 for 8^3)
    bool treeified = false;               // Java would have treeified a HashMap bin
    double coef_dc = 0.0;                 // the single DC group coefficient

    // ---- Java inverse (InverseDCT.java:87-133) ----
    std::vector<double> inv_coef;         // [cs * cs]  coefficients[n][k]

    // ---- fused-encode certification (fp32 kernel), per s = kx+ky+kz ----
    // |q_fp32 - q_java| <= A * enc_G[s] + enc_E[s], A = max |x - m| over the cube.
    float enc_rstep[kMaxS] = {};          // fp32(1/max(1,5s))
    float enc_G[kMaxS] = {};
    float enc_E[kMaxS] = {};
    // per-coefficient raw analysis results (exposed for tests)
    std::vector<double> enc_K;            // [cs] fp32 error bound per unit A
    std::vector<double> enc_L1;           // [cs] sum_n |basis|
    std::vector<double> enc_dev;          // [cs] grouping deviation bound (coef_g vs own coef)

    // ---- second certificate (8x8x8 encode, rare path): a coefficient the fp32 certificate leaves
    //      open is re-evaluated in fp64 as sum_n x_n * b[kz][z] b[ky][y] b[kx][x]; it is settled iff
    //      |q64 - rint(q64)| < enc_thr64[s] (q64 = v64 / step), else it goes to the exact Java fold ----
    double basis64[64] = {};              // orthonormal 8-point DCT-II basis [k][n], fp64
    double enc_thr64[kMaxS] = {};         // 0.5 - 2 * max_k E64_k per s (bound derivation: dct3d_plan.cpp)

    // ---- fused-decode certification (fp64 kernel) ----
    // |v_fp64 - v_java| <= L1_in * dec_G + dec_E, L1_in = sum |dequantised coefficient| over the cube;
    // a cube with L1_in >= dec_l1_max (|v| could reach 2^15) goes to the exact replay.
    double dec_G = 0.0, dec_E = 0.0;
    float dec_l1_max = 0.0f;

    // ---- inverse fp32-output / forward fp64-output kernels: informational bounds ----
    double fwd64_K = 0.0;                 // fp64 forward error per unit input magnitude
};

// Builds the plan for cube dims (cw, ch, cd).  Supported: cw = ch = 8, cd in {4, 8}.
// Returns false on unsupported dims.
bool build_plan(int cw, int ch, int cd, Plan& p);

}  // namespace dct3d
