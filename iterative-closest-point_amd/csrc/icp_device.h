// icp_device.h — device helpers shared by the engine's kernel files (icp_kernels.hip,
// icp_iter.hip): the workgroup sum, and the per-point arithmetic of the moment and transform
// passes, so that the fused small-cloud iteration (icp_iter.hip) rounds exactly like the
// separate kernels.  Compiled with -ffp-contract=off.
#pragma once

#include <hip/hip_runtime.h>

#include "icp_kernels.h"

namespace icp {

// Wave-then-workgroup sum of K doubles per thread; thread k < K of the workgroup writes
// out[k].  Fixed shuffle tree + fixed LDS order: deterministic.
template <int K>
__device__ __forceinline__ void block_sum_store(double (&a)[K], double *out)
{
    __shared__ double sh[kBlock / 64][K];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1)
#pragma unroll
        for (int k = 0; k < K; ++k) a[k] += __shfl_down(a[k], off, 64);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0)
#pragma unroll
        for (int k = 0; k < K; ++k) sh[wave][k] = a[k];
    __syncthreads();
    if (threadIdx.x < K) {
        const int k = threadIdx.x;
        out[k] = ((sh[0][k] + sh[1][k]) + sh[2][k]) + sh[3][k];
    }
}

// a[k] += row b's k-th value for this thread's rows b = t, t + kBlock, ... in that order (the
// reduce_kernel fold), four rows' loads issued before their sums: the same sums in the same
// order, one memory round trip per four rows instead of one per row
template <int K> __device__ __forceinline__ void fold_rows(const double *__restrict__ part, int nblocks, double (&a)[K])
{
    constexpr int kRows = 4;
    for (int b0 = threadIdx.x; b0 < nblocks; b0 += kRows * kBlock) {
        double v[kRows][K];
#pragma unroll
        for (int u = 0; u < kRows; ++u) {
            const int b = b0 + u * kBlock;
#pragma unroll
            for (int k = 0; k < K; ++k) v[u][k] = b < nblocks ? part[(size_t)b * K + k] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < kRows; ++u)
            if (b0 + u * kBlock < nblocks)
#pragma unroll
                for (int k = 0; k < K; ++k) a[k] += v[u][k];
    }
}

__device__ __forceinline__ void shifted_moment_terms(double px, double py, double pz, const double4 &m, double cp0,
                                                     double cp1, double cp2, double cy0, double cy1, double cy2,
                                                     double (&a)[17]);

// y_i = m[idx_i] (stored), then point i's terms of the one-pass moments around (cp, cy):
// sum (p - cp), sum (y - cy), sum (p - cp)(y - cy)^T, sum ||y - cy||^2, sum ||p - cp||^2
__device__ __forceinline__ void shifted_moment_point(int i, const int *__restrict__ idx,
                                                     const double4 *__restrict__ m4, const double *__restrict__ px,
                                                     const double *__restrict__ py, const double *__restrict__ pz,
                                                     double *__restrict__ yx, double *__restrict__ yy,
                                                     double *__restrict__ yz, double cp0, double cp1, double cp2,
                                                     double cy0, double cy1, double cy2, double (&a)[17],
                                                     const int *__restrict__ kpos = nullptr,
                                                     const double4 *__restrict__ m4kd = nullptr)
{
    const double4 m = kpos ? m4kd[kpos[i]] : m4[idx[i]]; // (kpos: the same point, kd-ordered copy)
    yx[i] = m.x;
    yy[i] = m.y;
    yz[i] = m.z;
    shifted_moment_terms(px[i], py[i], pz[i], m, cp0, cp1, cp2, cy0, cy1, cy2, a);
}

// point i's terms of the one-pass moments from its loaded p and y = m (shifted_moment_point's
// arithmetic, shared with the batched form of shifted_moments_kernel)
__device__ __forceinline__ void shifted_moment_terms(double px, double py, double pz, const double4 &m, double cp0,
                                                     double cp1, double cp2, double cy0, double cy1, double cy2,
                                                     double (&a)[17])
{
    const double p0 = px - cp0, p1 = py - cp1, p2 = pz - cp2;
    const double y0 = m.x - cy0, y1 = m.y - cy1, y2 = m.z - cy2;
    a[0] += p0;
    a[1] += p1;
    a[2] += p2;
    a[3] += y0;
    a[4] += y1;
    a[5] += y2;
    a[6] += p0 * y0;
    a[7] += p0 * y1;
    a[8] += p0 * y2;
    a[9] += p1 * y0;
    a[10] += p1 * y1;
    a[11] += p1 * y2;
    a[12] += p2 * y0;
    a[13] += p2 * y1;
    a[14] += p2 * y2;
    a[15] += (y0 * y0 + y1 * y1) + y2 * y2;
    a[16] += (p0 * p0 + p1 * p1) + p2 * p2;
}

// sR p + t in Eigen's column-sweep order (compute.cu:330-339, cpu.cc:33)
__device__ __forceinline__ void transform_point(const Xform &xf, double p0, double p1, double p2, double &q0,
                                                double &q1, double &q2)
{
    q0 = ((xf.sR[0] * p0 + xf.sR[1] * p1) + xf.sR[2] * p2) + xf.t[0];
    q1 = ((xf.sR[3] * p0 + xf.sR[4] * p1) + xf.sR[5] * p2) + xf.t[1];
    q2 = ((xf.sR[6] * p0 + xf.sR[7] * p1) + xf.sR[8] * p2) + xf.t[2];
}

// ||y - q||^2 (compute.cu:344-345)
__device__ __forceinline__ double residual2(double y0, double y1, double y2, double q0, double q1, double q2)
{
    const double e0 = y0 - q0, e1 = y1 - q1, e2 = y2 - q2;
    return (e0 * e0 + e1 * e1) + e2 * e2;
}

// f16 MFMA filter: queries whose scaled |coordinate| exceeds this are clamped and never certified
constexpr double kF16QueryClamp = 32000.0;
// every scaled model point b_s has |b_s| below this: the f16 image's scale puts each centred
// coordinate's magnitude below 2^12 (icp_set_model), and 2^12 sqrt 3 = 7094.6
constexpr double kF16ModelNormMax = 7095.0;

// Seeds of the seeded f16 filter from the previous correspondences prev[j] (exact fp64):
// s0 = G(m_prev) + 4 delta_s + 1 (the certificate window above that candidate's value, see
// nn_finalize_mfma16_kernel), rounded outward by 2^-20 and split into f16 hi/lo of -s0 / 2^14.
// seed of query p (unscaled fp64) from a model point m: packed f16 (hi | lo << 16) of -s0 / 2^14
__device__ __forceinline__ unsigned mfma16_seed_value(double p0, double p1, double p2, double m0, double m1,
                                                      double m2, double cx, double cy, double cz, double scale)
{
    const double a0 = fmin(fmax((p0 - cx) * scale, -kF16QueryClamp), kF16QueryClamp);
    const double a1 = fmin(fmax((p1 - cy) * scale, -kF16QueryClamp), kF16QueryClamp);
    const double a2 = fmin(fmax((p2 - cz) * scale, -kF16QueryClamp), kF16QueryClamp);
    const double b0 = (m0 - cx) * scale, b1 = (m1 - cy) * scale, b2 = (m2 - cz) * scale;
    const double bb = b0 * b0 + b1 * b1 + b2 * b2;
    const double G = bb - 2.0 * (a0 * b0 + a1 * b1 + a2 * b2);
    const double u = 0x1.0p-24;
    const double A = sqrt(a0 * a0 + a1 * a1 + a2 * a2), R = sqrt(bb);
    const double span = R * R + 2.0 * A * R;
    const double ds = 28.0 * u * R * R + 64.0 * u * A * R + 24.0 * u * (fabs(G) + 1e-3 * span) +
                      4.0 * u * (A + R) + 1e-3;
    double s0 = G + 4.0 * ds + 1.0;
    s0 += fabs(s0) * 0x1.0p-20;
    const double x = fmin(fmax(-s0 / 16384.0, -65000.0), 65000.0);
    const _Float16 hi = (_Float16)x;
    const _Float16 lo = (_Float16)(x - (double)hi);
    return (unsigned)__builtin_bit_cast(unsigned short, hi) | ((unsigned)__builtin_bit_cast(unsigned short, lo) << 16);
}

} // namespace icp
