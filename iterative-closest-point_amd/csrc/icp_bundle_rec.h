// icp_bundle_rec.h -- a query's operand record for the bundle filter (icp_bundle.hip): the
// constants, the bound operand (bundle_query_frag) and the record builder of its prep kernel.
#pragma once
#include "icp_device.h"
#include "icp_mfma16.h"

namespace icp {
namespace {

constexpr double kBQueryMax = 8192.0;                 // |a_k| range of the bundle operand
constexpr double kBSeedMax = 11000.0;                 // d' range of the bundle operand

// Query side of the bundle MFMA (see the file header): lane half h of query a (scaled,
// clamped), seed distance d' (already inflated).  Slots: h = 0: qx hi, lo, hi, qy hi, lo, hi,
// qz hi, lo; h = 1: qz hi, W hi, W lo, 4096, 4096, d hi, d lo, d hi, with
// W = (|q^|^2 - d'^2 - mu_q) / 4096.  kBqForced: V^ <= 0 for every bundle (a query outside the
// operand range); kBqNever: V^ > 0 for every bundle (a slot past the last query).
enum { kBqNormal = 0, kBqForced = 1, kBqNever = 2 };
__device__ __forceinline__ half8_t bundle_query_frag(const double a[3], double dq, int mode, int h)
{
    _Float16 xh, xl, yh, yl, zh, zl;
    split_f16(a[0], xh, xl);
    split_f16(a[1], yh, yl);
    split_f16(a[2], zh, zl);
    half8_t b;
    if (h == 0) {
        b[0] = xh; b[1] = xl; b[2] = xh; b[3] = yh;
        b[4] = yl; b[5] = yh; b[6] = zh; b[7] = zl;
        return b;
    }
    const double q0 = (double)xh + (double)xl, q1 = (double)yh + (double)yl, q2 = (double)zh + (double)zl;
    const double qq = (q0 * q0 + q1 * q1) + q2 * q2;
    const double mu = 0x1.0p-16 * (qq + dq * dq) + 0x1.0p-4;
    _Float16 wh, wl, dh, dl;
    split_f16((qq - dq * dq - mu) / 4096.0, wh, wl);
    split_f16(dq, dh, dl);
    if (mode != kBqNormal) { // forced: V^ < -6.7e7 for every bundle; never (no query): V^ > 6.7e7
        wh = mode == kBqForced ? (_Float16)-65504.0f : (_Float16)65504.0f;
        wl = (_Float16)0.0f;
        dh = (_Float16)0.0f;
        dl = (_Float16)0.0f;
    }
    b[0] = zh; b[1] = wh; b[2] = wl; b[3] = (_Float16)4096.0f;
    b[4] = (_Float16)4096.0f; b[5] = dh; b[6] = dl; b[7] = dh;
    return b;
}

struct BundleQuery {
    half8_t bound[2]; // bundle_query_frag, lane halves 0 / 1
    half8_t pair[2];  // query_frag (the seeded pair filter's operand)
};

// ---- the local-frame pair test (ICP_BUNDLE_LOCAL, the default with a scene in slot order) ----
// The pair test of the global f16 image evaluates G = |b|^2 - 2 a.b with |a|, |b| ~ 2^12: its
// error bound (nn_finalize_mfma16_kernel) is tens of scaled units, which leaves ~11% of the C4
// queries uncertified.  In the local form each 32-bundle block B has its own frame origin c_B
// (fp32, the midpoint of the block's box; R_B >= max |m - c_B| over its points) and its pair
// image holds m - c_B; the query operand is built per (group, fired block) from fl32(a) and
// c_B, and slots 14/15 carry |a_l|^2 - s0 instead of -s0.  The MFMA then sums
//     |m_l|^2 - 2 a_l.m_l + |a_l|^2 - s0  =  D - s0      (a_l = a - c_B, m_l = m - c_B)
// with every term of the order of (|a_l| + R_B)^2, not |a|^2: the same D values in every frame,
// so best / second compare across blocks as before, with the seed shift s0 in D units.
//
// Error bound (u = 2^-24, scaled units): for a pair with true D = |a - m|^2 (a = the clamped
// scaled query, m the scaled model point), R >= R_B, A' = sqrt(D) + R + u|a| + 1 >= |a_l|,
//   |D^ - (D - s0)| <= delta_local = 41u (A' + R)^2 + 30u s0 + 2 sqrt(D) E + E^2 + 2^-10
//                                    + 2^-23 (A' + R),   E = 5u A' + 4u R + u|a| + 2^-23,
// from: the model's hi/lo split and its |m_l|^2 slots (<= 12u R^2 + 2^-23 R + 2^-13); the
// shift slots: |a_l|^2 in fp32 (3.1u A'^2), minus s0 (u|w - s0|), the hi/lo split of
// (w - s0) / 2^14 (4u |w - s0| + 2^-11 for a subnormal lo), and |q'|^2 - |a_l|^2 for the split
// query q' (8u A'^2 + 2^-23 A'); the accumulation envelope of the f16 MFMA (24u sum |p|, as in
// nn_finalize_mfma16_kernel, sum |p| <= (A' + R)^2 + s0); and the position errors of the
// effective query and point, |q' - m' - (a - m)| <= E (fl32(a): u|a|; fl32(a - c_B): u A';
// the splits: 4u A' + 4u R + 2 x 2^-25 sqrt 3), which move |q' - m'|^2 off D by
// <= 2 sqrt(D) E + E^2.  The certificate and the seed use 1.25 delta_local + 1e-3.
__device__ __forceinline__ double delta_local(double D, double an, double R, double s0)
{
    const double u = 0x1.0p-24;
    const double sD = sqrt(fmax(D, 0.0));
    const double A = sD + R + u * an + 1.0;
    const double E = 5.0 * u * A + 4.0 * u * R + u * an + 0x1.0p-23;
    const double d = 41.0 * u * (A + R) * (A + R) + 30.0 * u * fabs(s0) + 2.0 * sD * E + E * E + 0x1.0p-10 +
                     0x1.0p-23 * (A + R);
    return 1.25 * d + 1e-3;
}

// The seed shift of the local pair test: s0 = D_s + 4 delta_local(2 D_s + 64) + 1 for the
// scaled seed distance D_s, rounded up to fp32.  The seed point's own value (<= D_s + delta)
// is then tracked, and a query whose second-nearest point lies beyond s0 certifies (the
// finalize needs s0 - b > 2 delta at the winner's D <= D_s + delta).
__device__ __forceinline__ float local_seed(double Ds, double an, double R)
{
    const double Dc = fmax(Ds, 0.0);
    const double s = Dc + 4.0 * delta_local(2.0 * Dc + 64.0, an, R, 2.0 * Dc + 64.0) + 1.0;
    float f = (float)s;
    if ((double)f < s) f = __uint_as_float(__float_as_uint(f) + 1u);
    return f;
}

// The local record's pair part: pair[0] = (fl32 a, s0) as the bits of a float4, pair[1] = 0.
__device__ __forceinline__ void bundle_local_pair(const double a[3], float s0, BundleQuery &r)
{
    const float4 v = make_float4((float)a[0], (float)a[1], (float)a[2], s0);
    r.pair[0] = __builtin_bit_cast(half8_t, v);
    r.pair[1] = half8_t{};
}

// The query operand half h of the local pair test in block frame c (fp32): a_l = fl32(a) - c
// in fp32, split hi/lo, and (|a_l|^2 - s0) / 2^14 split into slots 14/15 (clamped to the f16
// range: only a far pair of an out-of-range query gets there, and those are never certified).
__device__ __forceinline__ half8_t local_query_frag(const float4 aq, const float4 c, int h)
{
    const float lx = aq.x - c.x, ly = aq.y - c.y, lz = aq.z - c.z;
    const _Float16 xh = (_Float16)lx, yh = (_Float16)ly, zh = (_Float16)lz;
    const _Float16 xl = (_Float16)(lx - (float)xh), yl = (_Float16)(ly - (float)yh), zl = (_Float16)(lz - (float)zh);
    const _Float16 m2 = (_Float16)-2.0f;
    half8_t b;
    if (h == 0) {
        b[0] = m2 * xh; b[1] = m2 * xh; b[2] = m2 * xl; b[3] = m2 * yh;
        b[4] = m2 * yh; b[5] = m2 * yl; b[6] = m2 * zh; b[7] = m2 * zh;
        return b;
    }
    const float w = (lx * lx + ly * ly) + lz * lz;
    const float v = fminf(fmaxf((w - aq.w) * 0x1.0p-14f, -65000.0f), 65000.0f);
    const _Float16 sh = (_Float16)v, sl = (_Float16)(v - (float)sh);
    b[0] = m2 * zl; b[1] = (_Float16)4096.0f; b[2] = (_Float16)4096.0f; b[3] = m2 * xl;
    b[4] = m2 * yl; b[5] = m2 * zl; b[6] = sh; b[7] = sl;
    return b;
}

// Query j at p (unscaled fp64) with seed distance D = D64(p, m[prev j]) in the reference's
// arithmetic (compute.cu:112-117) and f16 seed sd (mfma16_seed_value): its record and
// raw = (p, j | sd << 32), what the certificate reads.  d' = (sqrt(D) S (1 + 2^-40) + e_q)
// (1 + 2^-20) + 2^-20 >= the seed distance in scaled units plus the query's own split error
// e_q (icp_bundle.hip's header); out-of-range queries are forced.
// local_r >= 0 (the local pair test, its R = max R_B): the pair part is bundle_local_pair's, and
// *s0_out receives the shift (the certificate's seed) instead of sd being used.
__device__ __forceinline__ void bundle_record(double p0, double p1, double p2, int j, double D, unsigned sd,
                                              double cx, double cy, double cz, double scale, BundleQuery &r,
                                              double4 &raw, double local_r = -1.0, float *s0_out = nullptr)
{
    double a[3];
    a[0] = fmin(fmax((p0 - cx) * scale, -kF16QueryClamp), kF16QueryClamp);
    a[1] = fmin(fmax((p1 - cy) * scale, -kF16QueryClamp), kF16QueryClamp);
    a[2] = fmin(fmax((p2 - cz) * scale, -kF16QueryClamp), kF16QueryClamp);
    const double eq = 0x1.0p-20 * ((fabs(a[0]) + fabs(a[1])) + fabs(a[2])) + 0x1.0p-22;
    const double dq = (sqrt(D) * scale * (1.0 + 0x1.0p-40) + 1e-300 + eq) * (1.0 + 0x1.0p-20) + 0x1.0p-20;
    const int mode = fabs(a[0]) <= kBQueryMax && fabs(a[1]) <= kBQueryMax && fabs(a[2]) <= kBQueryMax &&
                             dq <= kBSeedMax
                         ? kBqNormal
                         : kBqForced;
    raw = make_double4(p0, p1, p2, __longlong_as_double((long long)(((unsigned long long)sd << 32) | (unsigned)j)));
    r.bound[0] = bundle_query_frag(a, dq, mode, 0);
    r.bound[1] = bundle_query_frag(a, dq, mode, 1);
    if (local_r >= 0.0) {
        const double an = sqrt((a[0] * a[0] + a[1] * a[1]) + a[2] * a[2]);
        const float s0 = local_seed(D * scale * scale, an, local_r);
        bundle_local_pair(a, s0, r);
        if (s0_out) *s0_out = s0;
        return;
    }
    r.pair[0] = query_frag(a, 0, sd);
    r.pair[1] = query_frag(a, 1, sd);
}

// a padding slot's record: never fires (V^ > 0 for every bundle), index -1
__device__ __forceinline__ void bundle_never_record(BundleQuery &r, double4 &raw)
{
    const double a[3] = {0.0, 0.0, 0.0};
    raw = make_double4(0.0, 0.0, 0.0, __longlong_as_double(-1ll));
    r.bound[0] = bundle_query_frag(a, 0.0, kBqNever, 0);
    r.bound[1] = bundle_query_frag(a, 0.0, kBqNever, 1);
    r.pair[0] = query_frag(a, 0, 0u);
    r.pair[1] = query_frag(a, 1, 0u);
}

// The group bound: one column per 32-query group with the group's centre g^ (f16 hi/lo, the
// midpoint of its in-range queries' box) and D_g = max over them of (d'_q + |q^ - g^|) (rounded
// up), in bundle_query_frag's form.  |g^ - c^| > D_g + r' gives, for every query q of the group,
// |q^ - c^| >= |g^ - c^| - |q^ - g^| > d'_q + r', so a bundle the group excludes is excluded for
// each of its queries (same margins: V^ > 0 => V > 0).  A group with a kBqForced query is
// forced; one without in-range queries never fires.  Reductions over the 32 lanes of each half
// (lane and lane + 32 hold the same query).  Returns this lane's operand half for its group.
struct GroupBound {
    double g[3], D;
    int mode;
};
// the group of the 32-lane half `gh` (its lanes' queries q^ = hi + lo as the MFMA sees them,
// d', mode)
__device__ __forceinline__ GroupBound bundle_group_hat(const double q[3], double dq, int mode, int gh)
{
    const bool in = mode == kBqNormal;
    double lo3[3], hi3[3];
    for (int k = 0; k < 3; ++k) {
        lo3[k] = in ? q[k] : INFINITY;
        hi3[k] = in ? q[k] : -INFINITY;
    }
#pragma unroll
    for (int o = 16; o >= 1; o >>= 1)
        for (int k = 0; k < 3; ++k) {
            lo3[k] = fmin(lo3[k], __shfl_xor(lo3[k], o, 64));
            hi3[k] = fmax(hi3[k], __shfl_xor(hi3[k], o, 64));
        }
    const unsigned long long forced = __ballot(mode == kBqForced), normal = __ballot(in);
    const unsigned half_mask = gh ? (unsigned)(forced >> 32) : (unsigned)forced;
    const unsigned half_norm = gh ? (unsigned)(normal >> 32) : (unsigned)normal;
    double g[3];
    for (int k = 0; k < 3; ++k) {
        const double c = half_norm ? 0.5 * (lo3[k] + hi3[k]) : 0.0;
        _Float16 gh, gl;
        split_f16(c, gh, gl);
        g[k] = (double)gh + (double)gl;
    }
    const double e0 = q[0] - g[0], e1 = q[1] - g[1], e2 = q[2] - g[2];
    double D = in ? (dq + sqrt((e0 * e0 + e1 * e1) + e2 * e2) * (1.0 + 0x1.0p-48)) * (1.0 + 0x1.0p-48) : 0.0;
#pragma unroll
    for (int o = 16; o >= 1; o >>= 1) D = fmax(D, __shfl_xor(D, o, 64));
    int gmode = half_mask ? kBqForced : half_norm ? kBqNormal : kBqNever;
    if (gmode == kBqNormal && !(fabs(g[0]) <= kBQueryMax && fabs(g[1]) <= kBQueryMax && fabs(g[2]) <= kBQueryMax &&
                                D <= kBSeedMax))
        gmode = kBqForced;
    GroupBound r;
    for (int k = 0; k < 3; ++k) r.g[k] = g[k];
    r.D = D;
    r.mode = gmode;
    return r;
}
// group g = s / 32's bound from the record of this lane's slot s (lane = threadIdx.x & 63: the
// wave's two 32-lane halves are two groups); every lane of the wave takes part
__device__ __forceinline__ void bundle_group_store(const BundleQuery &rec, int s, int nslots, half8_t *__restrict__ gop,
                                                   double4 *__restrict__ gctr)
{
    const int lane = threadIdx.x & 63;
    const half8_t b0 = rec.bound[0], b1 = rec.bound[1];
    const double q[3] = {(double)b0[0] + (double)b0[1], (double)b0[3] + (double)b0[4], (double)b0[6] + (double)b0[7]};
    const double d = (double)b1[5] + (double)b1[6];
    const float w = (float)b1[1];
    const int mode = w == -65504.0f ? kBqForced : w == 65504.0f ? kBqNever : kBqNormal;
    const GroupBound gb = bundle_group_hat(q, d * (1.0 + 0x1.0p-20) + 0x1.0p-20, mode, lane >> 5);
    if ((lane & 31) < 2 && s < nslots) gop[(s >> 5) * 2 + (lane & 31)] = bundle_query_frag(gb.g, gb.D, gb.mode, lane & 31);
    if ((lane & 31) == 0 && s < nslots)
        gctr[s >> 5] = make_double4(gb.g[0], gb.g[1], gb.g[2],
                                    gb.mode == kBqNormal ? gb.D : gb.mode == kBqForced ? INFINITY : -1.0);
}

} // namespace
} // namespace icp
