// icp_step.hip — the per-iteration passes that end an ICP iteration's search (icp_run):
// the one-pass shifted moments (gpu.cc:98-104, :142) and the transform + residual (gpu.cc:71-74),
// each optionally ending in its own last workgroup with the fold and the Horn / error step
// (StepFold).  Compiled with IEEE semantics (unlike icp_kernels.hip's NN kernels, built with
// -fno-honor-nans): the error step's `err < threshold` must stay false for a NaN error, as in the
// reference's loop, and the Horn step must see NaN sums as they are.
#include <hip/hip_runtime.h>

#include "icp_bundle_rec.h"
#include "icp_device.h"
#include "icp_fold.h"
#include "icp_gridbox.h"
#include "icp_kernels.h"
#include "icp_mfma16.h"

#include <cstdlib>

namespace icp {
namespace {

// one pass around shifts near the centroids: the centred sums follow as
// S = sum (p - cp)(y - cy)^T - N dp dy^T etc. (horn_step), with N dp dy^T at rounding level
template <int kMomBatch, bool YIN, bool FOLD>
__global__ __launch_bounds__(kBlock, kMomBatch >= 8 ? 1 : 4) void shifted_moments_kernel(
    const int *__restrict__ idx, const double4 *__restrict__ m4, const double *__restrict__ px,
    const double *__restrict__ py, const double *__restrict__ pz, int n, double *__restrict__ yx,
    double *__restrict__ yy, double *__restrict__ yz, const IterState *__restrict__ st,
    double *__restrict__ partials, const int *__restrict__ kpos, const double4 *__restrict__ m4kd, StepFold fold)
{
    const bool frozen = st->done != 0; // a frozen (converged) ICP iteration: its sums are never used
    if (frozen && !FOLD) return; // (fused: every workgroup still arrives; the Horn step runs)
    const double cp0 = st->shift_p[0], cp1 = st->shift_p[1], cp2 = st->shift_p[2];
    const double cy0 = st->shift_y[0], cy1 = st->shift_y[1], cy2 = st->shift_y[2];
    double a[17];
#pragma unroll
    for (int k = 0; k < 17; ++k) a[k] = 0.0;
    // The thread's points i, i + G, i + 2G, ... (G = the grid's threads) in that order, as
    // shifted_moment_point takes them, but kMomBatch at a time with every load of the batch issued
    // before the first sum: at C4 a thread has four points, and one by one their dependent
    // (index -> model point) loads ran back to back.  Same sums, same order: bit-identical.
    const int G = gridDim.x * kBlock;
    for (int i0 = blockIdx.x * kBlock + threadIdx.x; i0 < (frozen ? 0 : n); i0 += kMomBatch * G) {
        int j[kMomBatch];
        if constexpr (!YIN) {
#pragma unroll
            for (int u = 0; u < kMomBatch; ++u) {
                const int i = i0 + u * G;
                j[u] = i < n ? (kpos ? kpos[i] : idx[i]) : 0;
            }
        }
        double4 m[kMomBatch];
        double qx[kMomBatch], qy[kMomBatch], qz[kMomBatch];
#pragma unroll
        for (int u = 0; u < kMomBatch; ++u) {
            const int i = i0 + u * G;
            const bool in = i < n;
            if constexpr (YIN) // (the search wrote y = m[idx]: the same values, streamed)
                m[u] = in ? make_double4(yx[i], yy[i], yz[i], 0.0) : make_double4(0.0, 0.0, 0.0, 0.0);
            else
                m[u] = in ? (kpos ? m4kd[j[u]] : m4[j[u]]) : make_double4(0.0, 0.0, 0.0, 0.0);
            qx[u] = in ? px[i] : 0.0;
            qy[u] = in ? py[i] : 0.0;
            qz[u] = in ? pz[i] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < kMomBatch; ++u) {
            const int i = i0 + u * G;
            if (i < n) {
                if constexpr (!YIN) {
                    yx[i] = m[u].x;
                    yy[i] = m[u].y;
                    yz[i] = m[u].z;
                }
                shifted_moment_terms(qx[u], qy[u], qz[u], m[u], cp0, cp1, cp2, cy0, cy1, cy2, a);
            }
        }
    }
    if constexpr (!FOLD) {
        block_sum_store<17>(a, partials + (size_t)blockIdx.x * 17);
        return;
    }
    // fused: reduce_horn_kernel's fold and Horn step in the last workgroup to arrive
    block_sum_publish<17>(a, partials + (size_t)blockIdx.x * 17);
    if (!last_arrival(fold.ticket)) return;
    __shared__ double s_sum[17];
    tail_fold<17>(partials, (int)gridDim.x, s_sum);
    if (threadIdx.x < 17) fold.sums[threadIdx.x] = s_sum[threadIdx.x];
    if (fold.step && threadIdx.x == 0) horn_step_body(s_sum, fold.N, fold.c[0], fold.c[1], fold.c[2], 1, fold.cnt, fold.s);
}

// a workgroup's count into *acc: one atomic, and only when it is not zero (a same-address
// atomic per workgroup would serialise ~1,000 of them a launch)
__device__ __forceinline__ void far_to_acc(int far, int *acc)
{
    __shared__ int s_far[kBlock / 64];
    for (int o = 32; o >= 1; o >>= 1) far += __shfl_xor(far, o, 64);
    if ((threadIdx.x & 63) == 0) s_far[threadIdx.x >> 6] = far;
    __syncthreads();
    if (threadIdx.x == 0) {
        int tot = 0;
        for (int w = 0; w < kBlock / 64; ++w) tot += s_far[w];
        if (tot) atomicAdd(acc, tot);
    }
}

// QOP: the form that also writes the next bundle search's slot records (sa.qop); without it the
// kernel carries none of their registers (the plain pass streams at a higher occupancy)
template <bool FOLD, bool QOP, int KB = 1>
__global__ __launch_bounds__(kBlock) void transform_err_kernel(
    double *__restrict__ px, double *__restrict__ py, double *__restrict__ pz,
    const double *__restrict__ yx, const double *__restrict__ yy, const double *__restrict__ yz,
    int n, Xform xfv, const Xform *__restrict__ xfd, const int *__restrict__ done, int write_p,
    float4 *__restrict__ p32, double *__restrict__ partials, SeedArgs sa, StepFold fold)
{
    // xfd / done (device-resident loop): the transform comes from the device Horn solve, and
    // nothing is applied once the loop has converged.  One load per workgroup, via LDS.
    __shared__ Xform sxf;
    __shared__ int sdone;
    if (threadIdx.x == 0) {
        sdone = done ? *done : 0;
        sxf = xfd ? *xfd : xfv;
    }
    __syncthreads();
    if (sdone && !FOLD) return; // (fused: every workgroup still arrives; the error step runs)
    const Xform xf = sxf;
    double a[1] = {0.0};
    int far = 0; // (sa.far_acc: this thread's moved points beyond sqrt(far_d2) of their correspondence)
    if (QOP && sa.qop && write_p) {
        // slot records (a scene in slot order): whole waves run to nslots (a multiple of 512; the
        // stride is a multiple of 64), so that each 32-slot group's lanes are all present for
        // its bound; the lanes past n build the padding's never-firing records -- every slot the
        // filter reads, so no earlier prep's padding is relied on
        for (int i = blockIdx.x * kBlock + threadIdx.x; i < sa.nslots; i += gridDim.x * kBlock) {
            BundleQuery r;
            if (i < n) {
                double q0, q1, q2;
                transform_point(xf, px[i], py[i], pz[i], q0, q1, q2);
                const double y0 = yx[i], y1 = yy[i], y2 = yz[i];
                a[0] += residual2(y0, y1, y2, q0, q1, q2);
                px[i] = q0;
                py[i] = q1;
                pz[i] = q2;
                if (p32)
                    p32[i] = make_float4((float)(q0 - xf.c[0]), (float)(q1 - xf.c[1]), (float)(q2 - xf.c[2]), 0.0f);
                const double dx = q0 - y0, dy = q1 - y1, dz = q2 - y2;
                const double d2 = (dx * dx + dy * dy) + dz * dz;
                far += sa.far_acc && seed_far(sa, q0, q1, q2, d2) ? 1 : 0;
                // (the seed distance too, as the plain form writes it: a later grid search -- of
                // this run, or of the next one carrying over -- reads it)
                if (sa.seedd) sa.seedd[i] = d2;
                double4 raw;
                if (sa.local_r >= 0.0) { // (the local pair test: the shift is the finalize's seed)
                    float s0;
                    bundle_record(q0, q1, q2, i, (dx * dx + dy * dy) + dz * dz, 0u, sa.c[0], sa.c[1], sa.c[2],
                                  sa.scale, r, raw, sa.local_r, &s0);
                    sa.seed16[i] = __float_as_uint(s0);
                } else {
                    const unsigned sd =
                        mfma16_seed_value(q0, q1, q2, y0, y1, y2, sa.c[0], sa.c[1], sa.c[2], sa.scale);
                    sa.seed16[i] = sd;
                    bundle_record(q0, q1, q2, i, (dx * dx + dy * dy) + dz * dz, sd, sa.c[0], sa.c[1], sa.c[2],
                                  sa.scale, r, raw);
                }
            } else {
                double4 raw;
                bundle_never_record(r, raw);
            }
            ((BundleQuery *)sa.qop)[i] = r;
            bundle_group_store(r, i, sa.nslots, (half8_t *)sa.gop, sa.gctr);
        }
        block_sum_store<1>(a, partials + blockIdx.x);
        if (sa.far_acc) far_to_acc(far, sa.far_acc);
        return;
    }
    // the thread's points i, i + G, i + 2G, ... in that order, KB at a time with every load of the
    // batch issued before the first transform (the same sums in the same order)
    const int G = gridDim.x * kBlock;
    for (int i0 = blockIdx.x * kBlock + threadIdx.x; i0 < (sdone ? 0 : n); i0 += KB * G) {
        double p0[KB], p1[KB], p2[KB], y0[KB], y1[KB], y2[KB];
#pragma unroll
        for (int u = 0; u < KB; ++u) {
            const int i = i0 + u * G;
            const bool in = i < n;
            p0[u] = in ? px[i] : 0.0;
            p1[u] = in ? py[i] : 0.0;
            p2[u] = in ? pz[i] : 0.0;
            y0[u] = in ? yx[i] : 0.0;
            y1[u] = in ? yy[i] : 0.0;
            y2[u] = in ? yz[i] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < KB; ++u) {
            const int i = i0 + u * G;
            if (i >= n) continue;
            double q0, q1, q2;
            transform_point(xf, p0[u], p1[u], p2[u], q0, q1, q2);
            a[0] += residual2(y0[u], y1[u], y2[u], q0, q1, q2);
            if (write_p) {
                px[i] = q0;
                py[i] = q1;
                pz[i] = q2;
                if (p32)
                    p32[i] = make_float4((float)(q0 - xf.c[0]), (float)(q1 - xf.c[1]), (float)(q2 - xf.c[2]), 0.0f);
                // the next seeded f16 search's seed: the new position against this iteration's
                // correspondence (y = m[idx], exactly what mfma16_seed_kernel would gather)
                if (sa.seed16)
                    sa.seed16[i] = mfma16_seed_value(q0, q1, q2, y0[u], y1[u], y2[u], sa.c[0], sa.c[1], sa.c[2],
                                                     sa.scale);
                if (sa.seedd || sa.far_acc) { // (bundle_prep_kernel's seed distance, in its arithmetic)
                    const double dx = q0 - y0[u], dy = q1 - y1[u], dz = q2 - y2[u];
                    const double d2 = (dx * dx + dy * dy) + dz * dz;
                    if (sa.seedd) sa.seedd[i] = d2;
                    far += sa.far_acc && seed_far(sa, q0, q1, q2, d2) ? 1 : 0;
                }
            }
        }
    }
    if constexpr (!FOLD) {
        block_sum_store<1>(a, partials + blockIdx.x);
        if (sa.far_acc) far_to_acc(far, sa.far_acc);
        return;
    }
    // fused: reduce_err_kernel's fold and error step in the last workgroup to arrive (the far
    // count is added first: the error step mirrors the loop state, far_acc included, to the host)
    if (sa.far_acc) far_to_acc(far, sa.far_acc);
    block_sum_publish<1>(a, partials + blockIdx.x);
    if (!last_arrival(fold.ticket)) return;
    __shared__ double loc[1];
    tail_fold<1>(partials, (int)gridDim.x, loc);
    if (threadIdx.x == 0) {
        fold.sums[kSumErr] = loc[0];
        if (fold.step)
            err_step_body(fold.sums, fold.N, fold.threshold, fold.max_iter, fold.err_trace, fold.s, fold.hflag,
                          fold.hticket, fold.h_state, fold.h_trace, true);
    }
}

} // namespace

void launch_shifted_moments(const int *idx, const double4 *m4, const double *px, const double *py,
                            const double *pz, int n, double *yx, double *yy, double *yz, const IterState *st_dev,
                            double *partials, hipStream_t st, const int *kpos, const double4 *m4kd, bool y_ready,
                            const StepFold &fold)
{
    // points of a thread whose loads are issued together (A/B: ICP_MOM_BATCH = 1 | 2 | 4; same
    // sums).  C4 (four points a thread): 23.5 / 20.5 / 21.2 us at 1 / 2 / 4 (profiles/r03bd/)
    static const int batch = [] {
        const char *e = getenv("ICP_MOM_BATCH");
        const int v = e ? atoi(e) : 2;
        return v == 1 || v == 4 || v == 8 ? v : 2;
    }();
#define MOMENTS(B, Y, F)                                                                                      \
    shifted_moments_kernel<B, Y, F><<<red_blocks(n), kBlock, 0, st>>>(idx, m4, px, py, pz, n, yx, yy, yz, st_dev, \
                                                                      partials, kpos, m4kd, fold)
#define MOMENTS_Y(B, Y)                                                                                       \
    do {                                                                                                      \
        if (fold.ticket) MOMENTS(B, Y, true);                                                                 \
        else MOMENTS(B, Y, false);                                                                            \
    } while (0)
    if (y_ready) {
        if (batch == 1) MOMENTS_Y(1, true);
        else if (batch == 4) MOMENTS_Y(4, true);
        else if (batch == 8) MOMENTS_Y(8, true);
        else MOMENTS_Y(2, true);
    } else {
        if (batch == 1) MOMENTS_Y(1, false);
        else if (batch == 4) MOMENTS_Y(4, false);
        else MOMENTS_Y(2, false);
    }
#undef MOMENTS_Y
#undef MOMENTS
}

void launch_transform_err(double *px, double *py, double *pz, const double *yx, const double *yy,
                          const double *yz, int n, Xform xf, int write_p, float4 *p32,
                          double *partials, hipStream_t st)
{
    transform_err_kernel<false, false><<<red_blocks(n), kBlock, 0, st>>>(px, py, pz, yx, yy, yz, n, xf, nullptr, nullptr,
                                                            write_p, p32, partials, SeedArgs{}, StepFold{});
}

// points of a thread whose loads are issued together in the plain transform (ICP_TR_BATCH = 1 | 2 |
// 4 | 8; the same sums).  C4 W = 1: 155.4-155.7 us per iteration at 2 against 157.3-159.0 at 1,
// 156.6-160.7 at 4 and 8; the W = 8 shard alike (profiles/r04z/trb_ab.txt)
static int transform_batch()
{
    static const int b = [] {
        const char *e = getenv("ICP_TR_BATCH");
        const int v = e ? atoi(e) : 2;
        return v == 1 || v == 4 || v == 8 ? v : 2;
    }();
    return b;
}

void launch_transform_err_dev(double *px, double *py, double *pz, const double *yx, const double *yy,
                              const double *yz, int n, const Xform *xf, const int *done, float4 *p32,
                              double *partials, const SeedArgs &sa, hipStream_t st, const StepFold &fold)
{
    // (the slot-record form ends without the fused step: its caller launches the error step)
    if (sa.qop)
        transform_err_kernel<false, true><<<red_blocks(n), kBlock, 0, st>>>(px, py, pz, yx, yy, yz, n, Xform{}, xf, done,
                                                                            1, p32, partials, sa, StepFold{});
    else if (fold.ticket)
        transform_err_kernel<true, false><<<red_blocks(n), kBlock, 0, st>>>(px, py, pz, yx, yy, yz, n, Xform{}, xf, done,
                                                                            1, p32, partials, sa, fold);
    else if (transform_batch() == 8)
        transform_err_kernel<false, false, 8><<<red_blocks(n), kBlock, 0, st>>>(px, py, pz, yx, yy, yz, n, Xform{}, xf,
                                                                                done, 1, p32, partials, sa, StepFold{});
    else if (transform_batch() == 4)
        transform_err_kernel<false, false, 4><<<red_blocks(n), kBlock, 0, st>>>(px, py, pz, yx, yy, yz, n, Xform{}, xf,
                                                                                done, 1, p32, partials, sa, StepFold{});
    else if (transform_batch() == 2)
        transform_err_kernel<false, false, 2><<<red_blocks(n), kBlock, 0, st>>>(px, py, pz, yx, yy, yz, n, Xform{}, xf,
                                                                                done, 1, p32, partials, sa, StepFold{});
    else
        transform_err_kernel<false, false><<<red_blocks(n), kBlock, 0, st>>>(px, py, pz, yx, yy, yz, n, Xform{}, xf,
                                                                             done, 1, p32, partials, sa, StepFold{});
}

} // namespace icp
