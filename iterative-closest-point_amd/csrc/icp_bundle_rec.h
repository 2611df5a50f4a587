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

// Query j at p (unscaled fp64) with seed distance D = D64(p, m[prev j]) in the reference's
// arithmetic (compute.cu:112-117) and f16 seed sd (mfma16_seed_value): its record and
// raw = (p, j | sd << 32), what the certificate reads.  d' = (sqrt(D) S (1 + 2^-40) + e_q)
// (1 + 2^-20) + 2^-20 >= the seed distance in scaled units plus the query's own split error
// e_q (icp_bundle.hip's header); out-of-range queries are forced.
__device__ __forceinline__ void bundle_record(double p0, double p1, double p2, int j, double D, unsigned sd,
                                              double cx, double cy, double cz, double scale, BundleQuery &r,
                                              double4 &raw)
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
